#!/bin/bash
# One GPU session of fixed steps (GPU box). Every step runs under its own time limit;
# the session stops at the first GPU fault, abort or timeout (exit codes other than
# 0/1; a plain test failure, 1, does not stop it). Logs: gpurun_out/run/<step>.log.
#
# Usage: bash tools/gpu_run.sh <step> ...
#   smoke        __graft_entry__.smoke()
#   tests        pytest -m gpu, stop at the first failure
#   tests_all    pytest -m gpu, every test
#   tests:<expr> pytest -m gpu -k <expr>
#   driver       bench.py as the driver runs it (--gpus 1 --steps 20 --warmup 5)
#   default      bench.py with no arguments
#   forcedist    bench.py under torch.distributed.run at world 1 (RCCL gather, configs_dist)
#   prof         the round's profile set (tools/prof_all.sh)
#   c4           configs[4] by lanes and hardware queues (bench.py --c4-only)
#   roctx        per-stage kernel time from the engine's roctx ranges (B = 16, 1)
#   pmcfit       PMC counter groups of the shipped small-batch fits (B = 16, 1)
#   fitdiag      small-batch fit: PMC passes of tools/blood_trace.py 16 and the stamped
#                tools/ubench/fit_diag over term-fold shapes (build fit_diag first)
#   twfdiag      the batch-wide tile-list fit (k_fit_sup_twf) against the (G, B) grids
#   timeline     rocprofv3 kernel timelines of one blood call at B = 1 and 16
#   peaksdiag    k_peaks fine against coarse chunks at B = 1, 4, 8, 16 (kernel traces)
#   synth:<B>    kernel stats of a synthetic device batch of B (tools/synth_batch.py)
#   c0diag       configs[0]: host/device breakdown (tools/c0_breakdown.py) and the phase
#                stamps of one pipeline (tools/stage_diag.py; the diag library first:
#                make -C metabodecon-rust_amd diag && cp .../build/libmdgpu_diag.so tools/ubench/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/run
log=gpurun_out/run/session.log
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $log
  timeout -k 10 "$t" "$@" > "gpurun_out/run/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $log
  tail -4 "gpurun_out/run/$name.log" | cut -c1-600 | tee -a $log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)" | tee -a $log; exit $rc; fi
  return 0
}
PYT=(python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread)
for step in "$@"; do
  case "$step" in
    smoke) run smoke 600 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 1200 "${PYT[@]}" -x ;;
    tests_all) run pytest_gpu 1200 "${PYT[@]}" ;;
    tests:*) run pytest_k 1200 "${PYT[@]}" -x -k "${step#tests:}" ;;
    driver) run driver_form 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    default) run default 600 python bench.py ;;
    forcedist) run forcedist 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --force-dist --steps 4 --warmup 1 --no-cpu-baseline ;;
    prof) run prof_all 1200 bash tools/prof_all.sh
      f=$(find gpurun_out/prof_q256 -name run_kernel_trace.csv | head -1)
      if [ -n "$f" ]; then run alone_q256 60 python tools/alone_kernels.py "$f" --out gpurun_out/bench_alone_q256.json \
          --command "rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu-baseline --no-configs --steps 6 --warmup 2 --verify 0"; fi ;;
    c4)
      cfgs=()
      for q in 4 32; do for l in 1 2 3 4 8 16; do
        [ $l -ge $q ] || cfgs+=("q${q}_l$l GPU_MAX_HW_QUEUES=$q MDGPU_LANES=$l --c4-only")
      done; done
      run c4 1200 bash tools/ab.sh c4 "${cfgs[@]}" ;;
    c4lanes)
      # configs[4]: one lane (one batch of 16) against two (8 + 8), three rounds
      ROUNDS=3 run c4lanes 1200 bash tools/ab.sh c4lanes "q4_l1 GPU_MAX_HW_QUEUES=4 MDGPU_LANES=1 --c4-only" \
        "q4_l2 GPU_MAX_HW_QUEUES=4 MDGPU_LANES=2 --c4-only" "q32_l1 GPU_MAX_HW_QUEUES=32 MDGPU_LANES=1 --c4-only" \
        "q32_l2 GPU_MAX_HW_QUEUES=32 MDGPU_LANES=2 --c4-only" ;;
    fitdiag)
      run pmc_fit 600 bash tools/pmc_fit.sh 16 16 992 tw7,tf,plain
      run fit_shapes_b16 120 tools/ubench/fit_diag 16 992 twf,twf1,tw7,s63.1.7@98,s63.2.7@16,s63.2.7@48,s63.1.7@16,s60.1.15@16,s60.1.15@50,s60.2.6@16,s63.2.3@16,s48.1.6@62,s63.1.9@98
      run fit_shapes_b8 120 tools/ubench/fit_diag 8 992 twf,twf1,s63.1.7@98,s63.2.7@32,s63.2.7@48,s60.1.15@32,s60.2.6@32
      run fit_shapes_b1 120 tools/ubench/fit_diag 1 992 twf,twf1,tf,s63.1.7@98,s63.2.7@48,s60.1.15@50 ;;
    twfdiag)
      run twf_b16 120 tools/ubench/fit_diag 16 992 tw7,twf,twf1,tw3s,twf3s,s63.1.7@98,s63.2.7@16,S63.1.3@98,S63.1.3@48,S63.1.7@98,S63.2.3@98
      run twf_b8 120 tools/ubench/fit_diag 8 992 tw7,tw3s,twf3s,S63.1.3@98
      run twf_b1 120 tools/ubench/fit_diag 1 992 tf,tw7,tw3s,twf3s,S63.1.3@98
      MDG_TW_G=768 run twf_b16_g768 120 tools/ubench/fit_diag 16 992 twf1
      MDG_TW_G=256 run twf_b16_g256 120 tools/ubench/fit_diag 16 992 twf,twf1
      MDG_TW_G=48 run twf_b1_g48 120 tools/ubench/fit_diag 1 992 twf,twf1 ;;
    timeline|timeline:*)
      # timeline:<fit kernel> forces MDG_FITSUP for the B = 16 trace
      fk=${step#timeline}; fk=${fk#:}
      for b in 1 16; do
        tag=bt$b${fk:+_$fk}
        if [ $b = 16 ] && [ -n "$fk" ]; then
          MDG_FITSUP=$fk run trace_$tag 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$tag -o run -- python3 tools/blood_trace.py $b
        else
          run trace_$tag 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$tag -o run -- python3 tools/blood_trace.py $b
        fi
        f=$(find gpurun_out/$tag -name run_kernel_trace.csv | head -1)
        if [ -n "$f" ]; then run timeline_$tag 60 python tools/blood_trace.py --summary "$f"; fi
      done ;;
    ab_r4)
      # round 4 small-batch defaults (twf1 fit, 4-point MSE tiles from B = 8) against the
      # round-3 choices, configs[4] alone; and the headline's MSE tile shape
      ROUNDS=2 run ab_c4 900 bash tools/ab.sh r4c4 "c4_new --c4-only" "c4_old MDG_FITSUP=tw7 MDG_MSE_NPT=2 --c4-only"
      ROUNDS=2 BENCH="--steps 8 --warmup 2" run ab_q 900 bash tools/ab.sh r4q "q_npt2" "q_npt4 MDG_MSE_NPT=4"
      cat gpurun_out/ab_r4c4/summary.txt gpurun_out/ab_r4q/summary.txt | tee -a $log ;;
    c4b) run c4_breakdown 300 python tools/c4_breakdown.py ;;
    exactmse)
      # the exact-order MSE option's cost: the headline queue and one spectrum at a time
      ROUNDS=2 BENCH="--steps 8 --warmup 2" run ab_exact 900 bash tools/ab.sh r4exact "q" "q_exact --exact-mse" \
          "b1 --mode stream --batch 1 --streams 1 --steps 40 --warmup 5" "b1_exact --mode stream --batch 1 --streams 1 --steps 40 --warmup 5 --exact-mse"
      cat gpurun_out/ab_r4exact/summary.txt | tee -a $log ;;
    fitb:*)
      # fitb:<B>: the fit kernels' launch durations in one blood call of B spectra
      b=${step#fitb:}
      for fk in ${FITB_KERNELS:-tw7 twf1 twf3s tf plain}; do
        tag=fit_b${b}_$fk
        MDG_FITSUP=$fk timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$tag -o run -- python3 tools/blood_trace.py $b > gpurun_out/run/$tag.log 2>&1 || { echo "STOP $tag"; exit 3; }
        f=$(find gpurun_out/$tag -name run_kernel_trace.csv | head -1)
        echo "== $tag $(python tools/blood_trace.py --summary "$f" | grep -E "fit|total" | awk '{s+=$4; n++} END {print n, s}')" | tee -a $log
      done ;;
    roctx)
      # stage attribution from the engine's roctx ranges (no hipEvents in the stream):
      # one blood call of 16 and of 1 spectra, kernel + HIP API + marker traces
      for b in 16 1; do
        tag=roctx_b$b
        MDG_ROCTX=1 run trace_$tag 180 rocprofv3 --kernel-trace --hip-trace --marker-trace --output-format csv -d gpurun_out/$tag -o run -- python3 tools/blood_trace.py $b
        run stages_$tag 60 python tools/roctx_stages.py gpurun_out/$tag --out gpurun_out/roctx_stages_b$b.json
      done ;;
    pmcfit)
      # PMC passes of the shipped small-batch fits (twf1 at B = 16, tf12 at B = 1 in
      # latency mode), summarised per batch (tools/pmc_groups.py)
      for b in 16 1; do
        run pmcfit_b$b 900 bash tools/pmc_fit.sh $b
        run pmcgroups_b$b 60 python tools/pmc_groups.py gpurun_out/pmcfit_b$b --out gpurun_out/pmc_fit_b$b.json
      done ;;
    msediag)
      # the MSE kernel at small batches: tile workgroups per spectrum and points per thread
      for v in "" "MDG_MSE_PARTS=128" "MDG_MSE_PARTS=64" "MDG_MSE_NPT=4" "MDG_MSE_NPT=4 MDG_MSE_PARTS=64"; do
        tag=mse_$(echo "$v" | tr ' =' '__')
        env $v MDG_FITSUP=twf1 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$tag -o run -- python3 tools/blood_trace.py 16 > gpurun_out/run/$tag.log 2>&1 || { echo "STOP $tag"; exit 3; }
        f=$(find gpurun_out/$tag -name run_kernel_trace.csv | head -1)
        echo "== $tag" | tee -a $log
        python tools/blood_trace.py --summary "$f" | grep -E "mse|total" | tee -a $log
        env $v timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag}_b1 -o run -- python3 tools/blood_trace.py 1 > gpurun_out/run/${tag}_b1.log 2>&1 || { echo "STOP $tag b1"; exit 3; }
        f=$(find gpurun_out/${tag}_b1 -name run_kernel_trace.csv | head -1)
        python tools/blood_trace.py --summary "$f" | grep -E "mse|select|total" | tee -a $log
      done ;;
    peaksdiag|peaksbig)
      # k_peaks' fine (staged) and coarse chunkings at small batches
      [ "$step" = peaksdiag ] && for B in 1 4 8 16; do for m in fine coarse; do
        tag=peaks_${m}_b$B
        MDG_PEAKS=$m timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$tag -o run -- python3 tools/blood_trace.py $B > gpurun_out/run/$tag.log 2>&1 || { echo "STOP $tag"; exit 3; }
        f=$(find gpurun_out/$tag -name run_kernel_trace.csv | head -1)
        echo "== $tag $(python tools/blood_trace.py --summary "$f" | grep -E "peaks")" | tee -a $log
      done; done
      for B in 64 256; do for m in fine coarse; do
        tag=peaks_${m}_s$B
        MDG_PEAKS=$m timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag -o run -- python3 tools/synth_batch.py $B 3 > gpurun_out/run/$tag.log 2>&1 || { echo "STOP $tag"; exit 3; }
        f=$(find gpurun_out/$tag -name run_kernel_stats.csv | head -1)
        echo "== $tag $(grep k_peaks "$f" | cut -c1-200)" | tee -a $log
      done; done ;;
    synth:*)
      # per-kernel stats of three pipelines of one synthetic device batch of B
      B=${step#synth:}; tag=synth_b$B
      timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag -o run -- python3 tools/synth_batch.py $B 3 > gpurun_out/run/$tag.log 2>&1 || { echo "STOP $tag"; exit 3; }
      f=$(find gpurun_out/$tag -name run_kernel_stats.csv | head -1)
      cut -d, -f1-4 "$f" | tee -a $log ;;
    decab)
      # compact rows decoded by the chain launch (default) against DMA + decode first
      for v in 1 0; do
        MDG_DEC_OVERLAP=$v run c0_dec$v 300 python tools/c0_breakdown.py 100
        for b in 1 16; do
          tag=dec${v}_b$b
          MDG_DEC_OVERLAP=$v timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$tag -o run -- python3 tools/blood_trace.py $b > gpurun_out/run/$tag.log 2>&1 || { echo "STOP $tag"; exit 3; }
          f=$(find gpurun_out/$tag -name run_kernel_trace.csv | head -1)
          echo "== $tag" | tee -a $log
          python tools/blood_trace.py --summary "$f" | grep -E "smooth|decode|total" | tee -a $log
        done
      done ;;
    hdab)
      # results written by the kernels into page-locked memory (default) against copies
      for v in 1 0 1 0; do MDG_HOST_DIRECT=$v run c0_hd$v 300 python tools/c0_breakdown.py 200; done ;;
    smallsets) run small_sets 600 python tools/small_sets.py ;;
    c0diag)
      run c0_breakdown 300 python tools/c0_breakdown.py 200
      run stage_diag_b1 120 python tools/stage_diag.py 1
      run stage_diag_b16 120 python tools/stage_diag.py 16 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done

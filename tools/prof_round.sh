set -e
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
bash tools/prof_session.sh trace b1 --streams 1 --steps 40
bash tools/prof_session.sh trace b256 --batch 256 --streams 1 --steps 2 --warmup 1
bash tools/prof_session.sh trace b4096_n65536 --batch 4096 --streams 1 --steps 1 --warmup 1 --n 65536 --peaks 1024 --hw-scale 2 --cap 2048
bash tools/prof_session.sh pmc b1 FETCH_SIZE --streams 1 --steps 5
bash tools/prof_session.sh pmc b1 WRITE_SIZE --streams 1 --steps 5
bash tools/prof_session.sh pmc b256 FETCH_SIZE --batch 256 --streams 1 --steps 1 --warmup 1
bash tools/prof_session.sh pmc b256 WRITE_SIZE --batch 256 --streams 1 --steps 1 --warmup 1

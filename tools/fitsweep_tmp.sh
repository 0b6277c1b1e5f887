export TMPDIR=/tmp; mkdir -p gpurun_out/fs3
L=metabodecon-rust_amd/metabodecon
for b in 16 8 1; do for v in pf1 pf2 pf3; do
  lib=$L/libmdgpu.so; [ $v = pf1 ] || lib=$L/libmdgpu_$v.so
  for g in 98 16; do
  MDGPU_LIB=$PWD/$lib MDGPU_ALLOW_STALE=1 MDG_TW_G=$g MDG_FITSUP=tw7 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fs3/${v}_g${g}_$b -o run -- python3 tools/blood_trace.py $b > gpurun_out/fs3/${v}_g${g}_$b.log 2>&1 || exit 1
  done
done; done

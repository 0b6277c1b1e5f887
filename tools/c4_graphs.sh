cd "${GRAFT_REPO_ROOT}"
for g in 0 1 0 1; do
  MDG_GRAPHS=$g timeout -k 10 200 python bench.py --configs 4 --no-cpu-baseline --steps 20 > gpurun_out/c4_$g.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('graphs', sys.argv[2], round(d['configs']['configs[4]']['value'],1), 'headline', round(d['value'],1))" gpurun_out/c4_$g.json $g
done

# A/B of library builds ab/libgpx_<name>.so with the full bench line (no side configs, no CPU baseline), alternating.
mkdir -p gpurun_out
for i in 1 2; do
  for v in "$@"; do
    GPX_LIB=$PWD/ab/libgpx_$v.so timeout -k 10 200 python bench.py --no-other-configs --no-cpu-baseline > gpurun_out/abB_${v}_$i.json 2>/dev/null || exit 1
  done
done
for f in gpurun_out/abB_*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', 'value %.4g' % d['value'], 'trmm %.3f ms frac %.4f' % (r['avg_launch_ms'], r['frac']), 'best', d['best'])"; done

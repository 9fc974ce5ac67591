export TMPDIR=/tmp
mkdir -p gpurun_out/bd
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --breakdown > gpurun_out/bd/bench.json 2> gpurun_out/bd/breakdown.txt || exit $?
for nb in 512 2048; do
  FVC_GDN_BLOCKS=$nb timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bd/gb_$nb.json 2>/dev/null || exit $?
  python -c "
import json; d=json.loads(open('gpurun_out/bd/gb_$nb.json').read().strip().splitlines()[-1]); h=d['hbm_kernels']
print('blocks=$nb', d['value'], {k: (h[k]['gb_per_s'], h[k]['ms_per_pframe']) for k in ('gdn', 'gdn+tap')})"
done

set -e
for v in "ASRX_DROPGEN_SIDE=1" "ASRX_DROPGEN_SIDE=0" "ASRX_DROPGEN_SIDE=0 ASRX_P3_XCD=1" "ASRX_DROPGEN_SIDE=1 ASRX_P3_XCD=1"; do
  for i in 1 2; do env $v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-probe 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', d['ms_per_step'])"; done
done

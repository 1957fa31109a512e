for k in 1 2 3; do for r in 1 4; do
  timeout -k 10 120 python -u bench.py --rounds $r --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rounds', $r, d['roofline']['kernel_ms_avg'], d['ms_per_step'])" || exit 1
done; done

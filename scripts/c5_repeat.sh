cd "$GRAFT_REPO_ROOT"
for i in 1 2 3; do timeout -k 10 120 python3 bench.py --config 5 --steps 2 --warmup 1 --no-cpu 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['roofline']['kernel_ms'], d['roofline']['gradients_per_launch_rank0'])"; done

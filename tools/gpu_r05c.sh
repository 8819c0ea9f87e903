set -euo pipefail
out=gpurun_out/r05c; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/t20 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dynamic --frames 5 > $out/t20.log 2>&1
ART_NO_LAUNCH_EVENT=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/t20n -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dynamic --frames 5 > $out/t20n.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/t2000 -o run -- python3 bench.py --steps 2000 --warmup 5 --no-cpu-baseline --no-dynamic --frames 5 > $out/t2000.log 2>&1
for i in 1 2 3; do timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dynamic --frames 5 | tail -1 | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('default 20', r['ms_per_step'])"; done
for i in 1 2 3; do ART_NO_LAUNCH_EVENT=1 timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dynamic --frames 5 | tail -1 | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('noev 20', r['ms_per_step'])"; done
for i in 1 2; do timeout -k 10 100 python bench.py --steps 5000 --warmup 5 --no-cpu-baseline --no-dynamic --frames 5 | tail -1 | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('default 5000', r['ms_per_step'])"; done
for i in 1 2; do ART_NO_LAUNCH_EVENT=1 timeout -k 10 100 python bench.py --steps 5000 --warmup 5 --no-cpu-baseline --no-dynamic --frames 5 | tail -1 | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('noev 5000', r['ms_per_step'])"; done
echo done

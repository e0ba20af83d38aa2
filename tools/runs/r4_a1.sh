# round 4, call a1: the horizon mode / value-definition build -- host CPU
# probe, the whole -m gpu suite, the driver's bench command, the secondary
# bench runs (--horizon 1000, --schedule reference, --dist init), smoke
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r4_a1}; mkdir -p $OUT; ROOT=$(pwd)
python3 - > $OUT/host.json <<'PY'
import json, os
d = {"os_cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}
for f in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpuset.cpus.effective", "/sys/fs/cgroup/memory.max"):
    try:
        d[f] = open(f).read().strip()
    except OSError as e:
        d[f] = str(e)
print(json.dumps(d))
PY
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --horizon 1000 > $OUT/bench_horizon.json 2> $OUT/bench_horizon.err || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --schedule reference > $OUT/bench_reference.json 2> $OUT/bench_reference.err || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --dist init > $OUT/bench_init.json 2> $OUT/bench_init.err || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
echo done > $OUT/ok

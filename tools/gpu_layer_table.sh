cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
OFLOW_TIMING_DUMP=gpurun_out/tdump.json timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_td.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_td.log | cut -c1-200

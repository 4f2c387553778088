#!/bin/bash
# GPU tests (-k $1), whole-step A/B base vs _build/ab_* ($2 rounds), then a kernel-stats
# profile of a short bench per library (top kernels by total time) into gpurun_out/abprof_*.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
bash tools/gpu_ab2.sh "$1" "" ${2:-2} || exit 1
for d in base optical_flow_amd/_build/ab_*; do
  if [ "$d" = base ]; then lib=optical_flow_amd/liboflow.so; else lib=$d/liboflow.so; fi
  [ -f $lib ] || continue
  n=$(basename $d)
  OFLOW_LIB=$lib timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abprof_$n -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --timing-steps 0 > gpurun_out/abprof_$n.log 2>&1 || exit 1
  echo "== $n"; python tools/kstats.py gpurun_out/abprof_$n/run_kernel_stats.csv 13 200 | grep -E "${3:-pack_many|bn_act|wgrad_reduce|warp_bwd|total}"
done

cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/stemwg
for v in 4 1 2 8 16 4; do
  echo "key10=$v"; timeout -k 10 120 python tools/conv_bench.py --reps 20 --only enc.conv1 --tune 10=$v 2>&1 | grep -v amdgpu.ids || exit 1
done

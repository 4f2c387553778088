cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
timeout -k 10 200 python tools/conv_bench.py --reps 10 --only "$1" 2>&1 | grep -v amdgpu.ids

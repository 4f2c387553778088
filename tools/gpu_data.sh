#!/bin/bash
# GPU check of the data path / flow pictures (SURVEY §8 f rows 1, 4): parity tests, then the
# data-path bench at B=8 and B=32, then the whole -m gpu suite.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/data
timeout -k 10 300 python -u -m pytest tests/test_gpu_data.py -x -v --timeout 120 --timeout-method thread > gpurun_out/data/pytest_data.log 2>&1 &&
timeout -k 10 300 python -u tools/data_bench.py --batch 8 --out gpurun_out/data/b8.json > gpurun_out/data/b8.log 2>&1 &&
timeout -k 10 300 python -u tools/data_bench.py --batch 32 --batches 20 --out gpurun_out/data/b32.json > gpurun_out/data/b32.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/data/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/data/pytest_data.log; cat gpurun_out/data/b8.json gpurun_out/data/b32.json 2>/dev/null; tail -3 gpurun_out/data/pytest_gpu.log
exit $rc

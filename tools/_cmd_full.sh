set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/t_full.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" gpurun_out/t_full.log | tail -3; grep -E "bf16 vs|1080x1920|RCCL|sharded" gpurun_out/t_full.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids

set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for E in "RAFT_CTX_SIDE=0" "AMD_SERIALIZE_KERNEL=3" "HIP_FORCE_DEV_KERNARG=0" "RAFT_EPI_STATS=0 RAFT_IN_NORM=0 RAFT_CONV_STEM=0"; do
  env $E timeout -k 10 300 python tools/diag_e2e4.py > gpurun_out/diag8.log 2>&1; rc=$?; echo "== $E rc=$rc"; grep -v amdgpu.ids gpurun_out/diag8.log | tail -3
  [ $rc -eq 0 ] || exit $rc
done

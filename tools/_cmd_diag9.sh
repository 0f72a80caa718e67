set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for E in "RAFT_CONV_STEM=0" "RAFT_EPI_STATS=0" "RAFT_IN_NORM=0" "RAFT_X=1"; do
  env $E timeout -k 10 300 python tools/diag_enc.py > gpurun_out/diag9e.log 2>&1; rc=$?; echo "== enc $E rc=$rc"; grep -v amdgpu.ids gpurun_out/diag9e.log | tail -1
  env $E timeout -k 10 300 python tools/diag_e2e4.py > gpurun_out/diag9.log 2>&1; rc=$?; echo "== e2e $E rc=$rc"; grep -v amdgpu.ids gpurun_out/diag9.log | tail -3
  [ $rc -eq 0 ] || exit $rc
done

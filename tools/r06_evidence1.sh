#!/bin/bash
# r06 evidence: per-conv SQ counters of the dominant conv (convc2 at B=1) with one (KS2=0) and two (KS2=1)
# compute waves per SIMD; the in-forward PMC passes (lookup HBM bytes, conv MFMA busy) and a config-2 forward
# trace of the current tree.  Each GPU step time-limited; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r06}
for KS in 0 1; do
  OUT=gpurun_out/pmcconv_convc2_ks$KS
  mkdir -p $OUT
  i=0
  for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU"; do
    i=$((i+1))
    RAFT_HALO_KS2=$KS timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/p$i -o run -- python tools/conv_bench.py 1 convc2 > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  done
  python tools/pmc_conv_summary.py $OUT conv_halo > gpurun_out/${TAG}_pmc_convc2_ks$KS.txt
  echo "## KS2=$KS"; cat gpurun_out/${TAG}_pmc_convc2_ks$KS.txt
done
RAFT_FUSE_CONVF1=1 PMC_OUT=gpurun_out PMC_ROUND=$TAG timeout -k 10 600 bash tools/pmc_forward.sh 1 > gpurun_out/pmc_$TAG.log 2>&1 || { tail -20 gpurun_out/pmc_$TAG.log; exit 1; }
tail -30 gpurun_out/pmc_$TAG.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fwd_$TAG -o run --output-format csv -- python tools/fwd_profile.py 1 440 1024 f16x3 > gpurun_out/fwd_$TAG.log 2>&1 || { tail -20 gpurun_out/fwd_$TAG.log; exit 1; }
python tools/phase_summary.py gpurun_out/fwd_$TAG/run_kernel_trace.csv > gpurun_out/${TAG}_forward_phases_config2.txt 2>&1
grep -E "forward span|encoder phase span|loop span" gpurun_out/${TAG}_forward_phases_config2.txt

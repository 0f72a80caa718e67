set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r06_base_bench.json 2> gpurun_out/r06_base_bench.err || { tail -20 gpurun_out/r06_base_bench.err; exit 1; }
cat gpurun_out/r06_base_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/fwd_r06base -o run --output-format csv -- python tools/fwd_profile.py 1 440 1024 f16x3 > gpurun_out/fwd_r06base.log 2>&1 || { tail -20 gpurun_out/fwd_r06base.log; exit 1; }
python tools/phase_summary.py gpurun_out/fwd_r06base/run_kernel_trace.csv > gpurun_out/r06base_forward_phases_config2.txt 2>&1
grep -E "forward span|encoder phase span|loop span" gpurun_out/r06base_forward_phases_config2.txt

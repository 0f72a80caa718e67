RAFT_HALO_CW8=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or update or gru or blocks or full_size or config or pair" > gpurun_out/t_cw8.log 2>&1; rc=$?; tail -3 gpurun_out/t_cw8.log; [ $rc -eq 0 ] || exit $rc
RAFT_HALO_CW8=1 timeout -k 10 200 python tools/fixed_cost.py > gpurun_out/fc_cw8.log 2>&1 && RAFT_HALO_CW8=0 timeout -k 10 200 python tools/fixed_cost.py > gpurun_out/fc_cw4.log 2>&1; grep fixed gpurun_out/fc_cw4.log gpurun_out/fc_cw8.log
./tools/ab_env.sh RAFT_HALO_CW8=0 RAFT_HALO_CW8=1

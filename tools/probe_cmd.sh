mkdir -p gpurun_out
run() {  # name, command...
  local n=$1; shift
  timeout -k 10 180 "$@" > gpurun_out/probe_$n.log 2>&1
  local rc=$?
  echo rc=$rc >> gpurun_out/probe_$n.log
  return $rc
}
run m_gred python -u tools/ddp_capture_probe.py 0 1 &&
run m_full python -u tools/ddp_capture_probe.py 1 1 &&
run graph_tests python -u -m pytest tests/test_gpu_graph.py -x -v --timeout 240 --timeout-method thread &&
UMAMD_DIST=1 run bench_dist1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --steps 10 --warmup 3 --no-roofline --no-cpu-baseline &&
run bench_n1 python bench.py --steps 10 --warmup 3 --no-roofline --no-cpu-baseline

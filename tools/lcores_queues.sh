# node_lcores (bench.py) under GPU_MAX_HW_QUEUES = 4 (HIP's default) / 8 / 16:
# one process each; the per-lcore graphs' streams share that many hardware queues
set -e
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 600 python -u -c "import sys; sys.path.insert(0,'.'); import bench, torch, json; torch.cuda.init(); print(json.dumps(bench.node_lcores(torch.device('cuda:0'))))" > gpurun_out/lcq_$q.json 2>> gpurun_out/lcq.err
done

"""How much of the per-step time is kernel, how much is event / launch gap (diagnostic)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench

dev = torch.device("cuda:0")
st = bench.build_state("c3", dev, 0, None)
stream = torch.cuda.current_stream(dev)
K = 40
for k in range(8):
    bench.run_step(st, stream, k)
torch.cuda.synchronize()
# (a) per-step events
evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
t = time.perf_counter()
for s in range(K):
    evs[s][0].record(stream); bench.run_step(st, stream, s); evs[s][1].record(stream)
torch.cuda.synchronize()
wa = (time.perf_counter() - t) / K * 1e3
pa = sum(a.elapsed_time(b) for a, b in evs) / K
# (b) one event pair around K steps
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t = time.perf_counter()
e0.record(stream)
for s in range(K):
    bench.run_step(st, stream, s)
e1.record(stream)
torch.cuda.synchronize()
wb = (time.perf_counter() - t) / K * 1e3
pb = e0.elapsed_time(e1) / K
# (c) events on a separate marker every 4 steps
print(f"per-step events: event ms {pa:.4f} wall ms/step {wa:.4f}")
print(f"one pair       : event ms/step {pb:.4f} wall ms/step {wb:.4f}")

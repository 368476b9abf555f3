import json, os, sys, time
import torch
sys.path.insert(0, os.getcwd())
import bench
dev = torch.device("cuda", 0); torch.cuda.set_device(dev)
w = bench.Workload("udp64", 0, 1, dev)
side = torch.cuda.Stream(device=dev)
cur = torch.cuda.current_stream()
def run(nstreams, steps=100):
    for i in range(steps):
        s = side if (nstreams == 2 and i % 2) else cur
        w.step(s.cuda_stream)
    torch.cuda.synchronize()
for _ in range(3): run(1, 100)
res = {1: [], 2: []}
for r in range(6):
    for ns in (1, 2) if r % 2 == 0 else (2, 1):
        torch.cuda.synchronize(); t0 = time.perf_counter(); run(ns, 200); el = time.perf_counter() - t0
        res[ns].append(round(w.n * 200 / el / 1e6, 1))
print(json.dumps({"placement": w.frames.pair_info, "streams1": res[1], "streams2": res[2]}))

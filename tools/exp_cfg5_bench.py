import os, sys, json, time
sys.path.insert(0, os.getcwd())
import torch
import bench
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
if len(sys.argv) > 1 and sys.argv[1] == "torchwork":
    x = torch.randint(0, 255, (1 << 30,), dtype=torch.uint8, device=dev)
    h = x.cpu().numpy()
    del x, h
out = bench.cfg5_proxy(torch, dev, 20, no_parity=True)
print(json.dumps({k: v for k, v in out.items() if k != "what"}), flush=True)

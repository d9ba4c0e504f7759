import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
mode = sys.argv[1]
import numpy as np
import xrs_amd
if mode == "call":
    x = xrs_amd.XRS(12, 4)
    v = [np.ones(4096, np.uint8) for _ in range(16)]
    x.encode(v)
import torch
print(mode, "is_available", torch.cuda.is_available(), "count", torch.cuda.device_count())
for l in open("/proc/self/maps"):
    if "amdhip64" in l or "hsa-runtime" in l:
        print(l.split()[-1]); 

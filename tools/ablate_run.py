"""Time the seal kernel of the library at NEB_LIB_PATH on the C2 batch (ablation study only)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from nebula_amd import workload as W
from nebula_amd.batch import DeviceBatch, install_keys
from nebula_amd.noiseutil import Engine
b = W.config(1)
eng = Engine(0, 16)
db = DeviceBatch(eng, b, install_keys(eng, b))
for _ in range(3): db.seal()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(20): db.seal()
e.record(); torch.cuda.synchronize()
print(os.environ.get("NEB_LIB_PATH"), "seal ms", s.elapsed_time(e) / 20)

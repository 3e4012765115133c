"""Time the seal kernel of the library at NEB_LIB_PATH on a config batch (ablation study only):
20 back-to-back seals, then 20 seal+open steps as bench.py runs them (kernel boundaries included)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from nebula_amd import workload as W
from nebula_amd.batch import DeviceBatch, install_keys
from nebula_amd.noiseutil import Engine
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 1
if cfg == 4:
    b = W.make_batch(1, 65536, 4096, sizes=(90, 576, 1300), ratio=(7, 4, 1))
elif cfg == 5:  # 61440 wave-groups: divides evenly over 16, 20 and 24 waves per CU
    b = W.make_batch(1, 983040, 1)
elif cfg == 8:  # C5 on one GPU: 1 Mi IMIX packets over 4096 keys
    b = W.config(4)
elif cfg in (6, 7):  # exactly 4 (6) or 16 (7) packets per key, 4096 keys: all tail / all full chunks
    per = 4 if cfg == 6 else 16
    b = W.make_batch(1, 4096 * per, 4096)
    b.desc["key_id"] = np.arange(b.n, dtype=np.uint32) % 4096
else:
    b = W.config(cfg)
eng = Engine(0, 4096)
db = DeviceBatch(eng, b, install_keys(eng, b))
for _ in range(3): db.seal()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(20): db.seal()
e.record(); torch.cuda.synchronize()
seal_ms = s.elapsed_time(e) / 20
db.open()
for _ in range(3):
    db.seal(); db.open()
torch.cuda.synchronize()
s.record()
for _ in range(20):
    db.seal(); db.open()
e.record(); torch.cuda.synchronize()
step_ms = s.elapsed_time(e) / 20
assert (db.status_host() == 0).all()
print(os.path.basename(os.environ.get("NEB_LIB_PATH", "default")), "seal ms %.4f" % seal_ms,
      "step ms %.4f" % step_ms, "pkts", b.n)

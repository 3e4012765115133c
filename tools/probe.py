"""Print what the engine sees on this box (device count, arch, runtime order effects)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nebula_amd import _lib as L  # noqa: E402

h = C.c_void_p()
rc = L.lib().neb_engine_create(0, 16, C.byref(h))
print("engine_create (library loaded before torch):", rc, L.lib().neb_last_error().decode())
if rc == 0:
    L.lib().neb_engine_destroy(h)
import torch  # noqa: E402

print("torch", torch.__version__, "cuda available", torch.cuda.is_available(), torch.cuda.get_device_name(0))
for m in ("libamdhip64",):
    for line in open("/proc/self/maps"):
        if m in line:
            print(line.split()[-1])
            break

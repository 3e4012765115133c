"""Does hipStreamGetId name a stream uniquely? Creates and destroys streams in turn (the allocator may
hand a new stream the old one's address) and prints handle and id of each: engine.cpp StreamTag keys
its skip of the cross-stream wait on the pair."""
import ctypes
import json

hip = ctypes.CDLL("libamdhip64.so")
rows = []
for k in range(6):
    s = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
    sid = ctypes.c_ulonglong()
    assert hip.hipStreamGetId(s, ctypes.byref(sid)) == 0
    rows.append({"k": k, "handle": hex(s.value or 0), "id": sid.value})
    assert hip.hipStreamDestroy(s) == 0
handles = [r["handle"] for r in rows]
ids = [r["id"] for r in rows]
print(json.dumps({"streams": rows, "handles_reused": len(set(handles)) < len(handles),
                  "ids_unique": len(set(ids)) == len(ids)}))

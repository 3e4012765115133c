"""Condense a tools/profile.sh `lds` counter pass into profiles/pmc_busy.json: per kernel, the
fraction of its CU-busy cycles the LDS array was busy (SQ_LDS_IDX_ACTIVE / SQ_BUSY_CU_CYCLES) and
the VALU was busy (SQ_INSTS_VALU x 4 cycles per wave64 op over the SIMDs, per CU / the same span).
These are the resources that bound the AEAD kernels; bench.py reports them
beside the HBM roofline. usage: python tools/pmc_busy.py profiles/<tag> [more tags...]"""
import json
import os
import re
import sys

CUS, SIMDS_PER_CU, VALU_CYCLES = 256, 4, 2


def short(name):
    m = re.search(r"neb::(\w+<[^>]*>|\w+)\(", name)
    return m.group(1) if m else name


def main():
    out = {"source": [], "kernels": {}}
    for d in sys.argv[1:]:
        lds = json.load(open(os.path.join(d, "pmc_lds.json")))
        out["source"].append(d)
        for k, c in lds.items():
            busy = c.get("SQ_BUSY_CU_CYCLES")
            if not busy or "neb::" not in k:
                continue
            per_cu = busy / CUS
            out["kernels"][short(k)] = {
                "lds_busy": round(c["SQ_LDS_IDX_ACTIVE"] / busy, 3),
                "valu_busy": round(c["SQ_INSTS_VALU"] / (CUS * SIMDS_PER_CU) * VALU_CYCLES / per_cu, 3),
                "source": os.path.join(d, "pmc_lds.json"),
            }
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "pmc_busy.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out["kernels"], indent=1))


if __name__ == "__main__":
    main()

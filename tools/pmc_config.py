"""Record one bench config's counter passes in profiles/pmc_configs.json, keyed by config (not by
kernel name: C3 and C5 run the same mixed-key kernel, with different traffic).

From a profiles/<tag> directory written by tools/pmc_summary.py (pmc_fetch.json, pmc_write.json,
pmc_lds.json, trace_kernel_stats.csv) it takes, for the config's dominant kernel (the seal launch):
  hbm_bytes_per_launch = the memory-side requests by size when the tag has them (pmc_req.json,
                         pmc_wreq.json: 32/64/128 B x TCC_EA0_RDREQ_32B/_64B/_128B and 64 B x
                         TCC_EA0_WRREQ_64B + 32 B x the other write requests), else
                         2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes; MI355X_MICROARCH.md §HBM: on
                         gfx950 FETCH_SIZE reports half the bytes of 16 B/lane streaming reads)
  lds_busy  = SQ_LDS_IDX_ACTIVE / SQ_BUSY_CU_CYCLES
  valu_busy = VALU issue cycles per SIMD over the CU-busy cycles: a wave64 VALU instruction takes
              one quad-cycle (4 cycles), two VOP1/VOP2 of two waves share one (SQ_ACTIVE_INST_VALU2
              counts the second), so 4 x (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2) / 4 SIMDs per CU
              (tools/valu_issue.py); passes without VALU2 count no co-issue
  mean_ns   = the kernel's rocprof mean duration (the same passes' kernel trace)
usage: python tools/pmc_config.py CONFIG KERNEL_SUBSTRING profiles/<tag> [profiles/<tag with the lds pass>]
   e.g. python tools/pmc_config.py C3 "gcm_chunk_kernel<false>" profiles/r3q_c3 profiles/r3_c3
"""
import csv
import json
import os
import sys

CUS, SIMDS_PER_CU, VALU_CYCLES = 256, 4, 4
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def pick(d, sub):
    hits = [k for k in d if sub in k]
    if not hits:
        raise SystemExit(f"no kernel matching {sub!r} in {sorted(d)}")
    return d[sorted(hits, key=len)[0]]


def main():
    cfg, sub, tag = sys.argv[1:4]
    lds_tag = sys.argv[4] if len(sys.argv) > 4 else tag
    load = lambda n, t=tag: json.load(open(os.path.join(t, f"pmc_{n}.json")))  # noqa: E731
    f, w = pick(load("fetch"), sub), pick(load("write"), sub)
    ent = {
        "kernel": sub,
        "fetch_size_kib": round(f["FETCH_SIZE"], 1),
        "write_size_kib": round(w["WRITE_SIZE"], 1),
        "hbm_bytes_per_launch": int(2 * f["FETCH_SIZE"] * 1024 + w["WRITE_SIZE"] * 1024),
        "source": os.path.relpath(tag, ROOT),
    }
    try:
        rq, wq = pick(load("req"), sub), pick(load("wreq"), sub)
        rd = 32 * rq["TCC_EA0_RDREQ_32B"] + 64 * rq["TCC_EA0_RDREQ_64B"] + 128 * rq["TCC_EA0_RDREQ_128B"]
        wr = 64 * wq["TCC_EA0_WRREQ_64B"] + 32 * (wq["TCC_EA0_WRREQ"] - wq["TCC_EA0_WRREQ_64B"])
        ent["read_bytes_req"], ent["write_bytes_req"] = int(rd), int(wr)
        ent["rdreq_128b_frac"] = round(rq["TCC_EA0_RDREQ_128B"] / max(1.0, rq["TCC_EA0_RDREQ"]), 4)
        ent["hbm_bytes_per_launch"] = int(rd + wr)
        ent["hbm_bytes_basis"] = "request sizes (TCC_EA0_RDREQ_32B/64B/128B, TCC_EA0_WRREQ/_64B)"
    except (OSError, KeyError, SystemExit):
        ent["hbm_bytes_basis"] = "2 x FETCH_SIZE + WRITE_SIZE"
    if lds_tag != tag:
        ent["lds_source"] = os.path.relpath(lds_tag, ROOT)
    try:
        lds = pick(load("lds", lds_tag), sub)
        busy = lds["SQ_BUSY_CU_CYCLES"]
        ent["lds_busy"] = round(lds["SQ_LDS_IDX_ACTIVE"] / busy, 3)
        issued = lds["SQ_INSTS_VALU"] - lds.get("SQ_ACTIVE_INST_VALU2", 0.0)
        ent["valu_busy"] = round(issued / (CUS * SIMDS_PER_CU) * VALU_CYCLES / (busy / CUS), 3)
        ent["valu_coissue_counted"] = "SQ_ACTIVE_INST_VALU2" in lds
    except (OSError, KeyError, SystemExit):
        pass
    stats = os.path.join(tag, "trace_kernel_stats.csv")
    if os.path.exists(stats):
        for r in csv.DictReader(open(stats)):
            if sub in r["Name"]:
                ent["mean_ns"] = round(float(r["AverageNs"]), 1)
                break
    path = os.path.join(ROOT, "profiles", "pmc_configs.json")
    allc = json.load(open(path)) if os.path.exists(path) else {}
    allc[cfg] = ent
    json.dump(allc, open(path, "w"), indent=1, sort_keys=True)
    print(cfg, json.dumps(ent))


if __name__ == "__main__":
    main()

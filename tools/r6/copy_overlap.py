"""Host-staged pipeline timeline from a rocprofv3 memory-copy + kernel trace (csv): per call, the
copy-in (SDMA H2D), kernel and copy-back (blit kernel or SDMA D2H) intervals, how long each
direction is busy, how much of the call has both directions in flight, and the gaps before each
copy-in with what ended just before them.

usage: python tools/r6/copy_overlap.py <prefix>_memory_copy_trace.csv <prefix>_kernel_trace.csv
"""
import csv
import sys


def load(mc_path, kt_path):
    ev = []
    for r in csv.DictReader(open(mc_path)):
        d = "in" if "HOST_TO_DEVICE" in r["Direction"] else "back"
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), d))
    for r in csv.DictReader(open(kt_path)):
        name = r["Kernel_Name"]
        kind = "back" if "copyBuffer" in name else "kernel"
        if "key_setup" in name:
            continue
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind))
    ev.sort()
    return ev


def calls(ev, idle_ns=100_000):
    out, cur, end = [], [], None
    for e in ev:
        if end is not None and e[0] - end > idle_ns:
            out.append(cur)
            cur = []
        cur.append(e)
        end = e[1] if end is None else max(end, e[1])
    if cur:
        out.append(cur)
    return out


def busy(iv):
    iv = sorted(iv)
    tot, s0, e0 = 0, None, None
    for s, e in iv:
        if e0 is None or s > e0:
            if e0 is not None:
                tot += e0 - s0
            s0, e0 = s, e
        else:
            e0 = max(e0, e)
    if e0 is not None:
        tot += e0 - s0
    return tot


def both(a, b):
    tot = 0
    for s1, e1 in a:
        for s2, e2 in b:
            tot += max(0, min(e1, e2) - max(s1, s2))
    return tot


def main():
    ev = load(sys.argv[1], sys.argv[2])
    cs = calls(ev)
    print("call  span_us  in_busy  back_busy  both  kernel_busy  in_gaps(us: after what)")
    for c in cs[-8:]:
        t0, t1 = c[0][0], max(e[1] for e in c)
        ins = [(s, e) for s, e, k in c if k == "in"]
        backs = [(s, e) for s, e, k in c if k == "back"]
        ks = [(s, e) for s, e, k in c if k == "kernel"]
        gaps = []
        for i in range(1, len(ins)):
            g = ins[i][0] - ins[i - 1][1]
            if g > 30_000:
                before = [k for s, e, k in c if ins[i][0] - 10_000 <= e <= ins[i][0]]
                gaps.append(f"{g / 1e3:.0f}:{'/'.join(before) or '-'}")
        print(f"{len(ins):4d} {(t1 - t0) / 1e3:8.1f} {busy(ins) / 1e3:8.1f} {busy(backs) / 1e3:9.1f} "
              f"{both(ins, backs) / 1e3:6.1f} {busy(ks) / 1e3:11.1f}  {' '.join(gaps)}")


if __name__ == "__main__":
    main()

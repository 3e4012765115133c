"""Median per-dispatch duration (µs) of every kernel in rocprofv3 kernel-trace CSVs.

usage: python tools/trace_sched.py <trace dir or csv> ...
"""
import collections
import csv
import glob
import os
import sys


def medians(path):
    files = [path] if path.endswith('.csv') else glob.glob(os.path.join(path, '**', '*kernel_trace.csv'), recursive=True)
    d = collections.defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            d[r['Kernel_Name'].split('(')[0]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    return {k: (len(v), sorted(v)[len(v) // 2]) for k, v in d.items()}


if __name__ == '__main__':
    for p in sys.argv[1:]:
        print(p)
        for k, (n, m) in sorted(medians(p).items(), key=lambda kv: -kv[1][1]):
            print(f'  {m:9.2f} us  x{n:<4d} {k}')

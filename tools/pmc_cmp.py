#!/usr/bin/env python3
"""Mean PMC counters per variant for one kernel from tools/ablate_gpu.sh output."""
import collections, csv, sys
kern = sys.argv[1] if len(sys.argv) > 1 else 'gcm_single_kernel<false>'
for v in open('build_abl/variants.txt').read().split():
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f'gpurun_out/ablate/{v}/{v}_counter_collection.csv')):
        if kern in r['Kernel_Name']:
            d[r['Counter_Name']].append(float(r['Counter_Value']))
    print(f"{v:8s}", ' '.join(f"{k.replace('SQ_','')}={sum(x)/len(x)/1e6:.2f}M" for k, x in sorted(d.items())))

"""Summarise rocprofv3 --pmc CSVs per (kernel, grid) -> mean counter values."""
import collections
import csv
import sys

res = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r['Kernel_Name'].split('(')[0].replace('aec::', '')
        if 'rocclr' in k:
            continue
        res[(k, int(r['Grid_Size']))][r['Counter_Name']].append(float(r['Counter_Value']))
for (k, g), d in sorted(res.items()):
    print(k, g, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})

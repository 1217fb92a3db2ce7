"""Per-kernel duration stats from a rocprofv3 kernel trace, grouped by (name, grid size)."""
import collections
import csv
import sys

r = list(csv.DictReader(open(sys.argv[1])))
grp = collections.defaultdict(list)
for x in r:
    key = (x['Kernel_Name'][:70], int(x['Grid_Size_X']) * int(x['Grid_Size_Y']))
    grp[key].append((int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1e3)
rows = sorted(grp.items(), key=lambda kv: -sum(kv[1]))
for (name, grid), d in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    d = sorted(d)
    print('%-70s grid %8d  n %5d  median %8.1f us  total %8.1f us' % (name, grid, len(d), d[len(d) // 2], sum(d)))

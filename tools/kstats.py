import csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(x['TotalDurationNs']) for x in r)
for x in r[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print('%-100s %6s %10.1f us %6.2f%%' % (x['Name'][:100], x['Calls'], float(x['AverageNs'])/1e3, float(x['Percentage'])))
print('total GPU time %.1f ms' % (tot / 1e6))

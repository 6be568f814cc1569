import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows: print('%-70s %6s %10.1f us avg %10.1f total' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e3))

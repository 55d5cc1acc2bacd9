import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n=r['Name'].replace('(anonymous namespace)::','').replace('void ','').split('(')[0]
    if n.startswith('__amd'): continue
    print(f"{n:45s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:8.2f} min {float(r['MinNs'])/1e3:7.2f} max {float(r['MaxNs'])/1e3:7.2f}")

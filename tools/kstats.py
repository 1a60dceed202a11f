import csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(x['TotalDurationNs']) for x in r)
print(f"total {tot/1e6:.1f} ms")
for x in r[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f"{x['Name'][:70]:70s} {x['Calls']:>5} {float(x['TotalDurationNs'])/1e6:9.2f} ms {float(x['AverageNs'])/1e3:9.1f} us {x['Percentage'][:5]}")

import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.Counter()
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'][:40]
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
        calls[(k, r['Counter_Name'])] += 1
names = sorted(agg, key=lambda k: -agg[k].get('SQ_WAVE_CYCLES', agg[k].get('FETCH_SIZE', 0)))
for k in names:
    print(k, {c: f"{v:.3g}" for c, v in agg[k].items()})

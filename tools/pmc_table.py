"""Per-dispatch counter table for tamd_exec from rocprofv3 counter_collection CSVs."""
import csv, collections, sys
for p in sys.argv[1:]:
    rows = [r for r in csv.DictReader(open(p + '/run_counter_collection.csv')) if r['Kernel_Name'].startswith('tamd_exec')]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for r in rows:
        agg[r['Dispatch_Id']][r['Counter_Name']] += float(r['Counter_Value'])
        dur[r['Dispatch_Id']] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    ds = sorted(agg, key=int)
    names = sorted({k for d in ds for k in agg[d]})
    print(p, ' '.join(n[:22].rjust(22) for n in names), 'us')
    for d in ds:
        print(d.rjust(4), ' '.join(f'{agg[d][n]:22.0f}' for n in names), f'{dur[d]:.1f}')

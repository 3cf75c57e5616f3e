"""Per-launch tamd_exec durations from a rocprofv3 kernel trace, grouped per program (4 levels)."""
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/*kernel_trace.csv')[0]
rows = [r for r in csv.DictReader(open(f)) if r['Kernel_Name'].startswith('tamd_exec')]
d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows]
per = int(sys.argv[2]) if len(sys.argv) > 2 else 4
for i in range(0, len(d), per):
    print(' '.join(f'{x:7.1f}' for x in d[i:i + per]), f'| sum {sum(d[i:i+per]):7.1f}')
print('avg', sum(d) / len(d), 'n', len(d))

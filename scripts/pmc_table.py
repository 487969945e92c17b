"""Per-kernel sums of rocprofv3 counter-collection CSVs (one or more pass dirs), averaged per dispatch:
python scripts/pmc_table.py gpurun_out/pmc_TAG_1 gpurun_out/pmc_TAG_2 ... [--kernel SUBSTR]"""
import collections, csv, glob, sys
args = [a for a in sys.argv[1:] if not a.startswith('--')]
ksub = ''
if '--kernel' in sys.argv:
    ksub = sys.argv[sys.argv.index('--kernel') + 1]
    args = [a for a in args if a != ksub]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for d in args:
    for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name'].split('(')[0]
            if ksub and ksub not in k:
                continue
            tot[k][r['Counter_Name']] += float(r['Counter_Value'])
            disp[k].add((f, r['Dispatch_Id']))
for k, c in tot.items():
    n = max(1, len(disp[k]) // max(1, len(args)))
    print(k[:70], 'dispatches/pass', n)
    for name, v in sorted(c.items()):
        print('   %-32s %16.0f per dispatch' % (name, v / n))

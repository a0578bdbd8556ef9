import csv, glob, sys, collections, os
root=sys.argv[1]
for d in sorted(glob.glob(root+'/*_p*')):
    f=glob.glob(d+'/**/*counter_collection.csv', recursive=True)
    if not f: print(d,'no csv'); continue
    agg=collections.defaultdict(float); n=collections.Counter()
    for row in csv.DictReader(open(f[0])):
        if 'kno' not in row.get('Kernel_Name','') or 'k_trace' not in row.get('Kernel_Name',''): continue
        agg[row['Counter_Name']]+=float(row['Counter_Value']); n[row['Counter_Name']]+=1
    print(os.path.basename(d), {k: round(v/ max(1,n[k]),1) for k,v in agg.items()})

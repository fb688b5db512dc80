import csv, glob, collections, os
res = collections.defaultdict(list)
for d in sorted(glob.glob('gpurun_out/plansplit/*_*_*/')):
    name = os.path.basename(d.rstrip('/'))
    c, v, rep = name.split('_')
    f = glob.glob(d + '*kernel_trace.csv')
    if not f: continue
    rows = list(csv.DictReader(open(f[0])))
    tot = collections.defaultdict(float); nb = 0
    for r in rows:
        k = r['Kernel_Name']
        dur = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
        for key in ('k_rewalk_scan_lean', 'k_rewalk_plan_lean', 'k_rewalk_sorted'):
            if key in k:
                tot[key] += dur
        if 'k_rewalk_sorted' in k: nb += 1
    per = {k: round(v2 / nb, 3) for k, v2 in tot.items()}
    res[(c, v)].append((rep, nb, per, round(sum(tot.values()) / nb, 3)))
for k in sorted(res):
    for x in res[k]: print(k, x)

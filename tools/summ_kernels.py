import csv,glob,sys
f=glob.glob(sys.argv[1]+'/*kernel_stats.csv')[0]
for r in csv.DictReader(open(f)):
    n=r['Name']; n=n.replace('(anonymous namespace)::','').replace('void ','').replace('lhpc::','')
    if 'at::' in n: continue
    print(f"{n.split('(')[0][:60]:60s} calls {r['Calls']:>4s} avg_us {float(r['AverageNs'])/1e3:9.1f} total_ms {float(r['TotalDurationNs'])/1e6:8.2f}")

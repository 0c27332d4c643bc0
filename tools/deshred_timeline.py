"""Timeline of the last composed deshred in a rocprofv3 --kernel-trace --hip-trace run
(bench_shredder.py under the profiler): kernels with a host gap > 20 us or a duration > 300 us,
the span from shred_deserialize to pipe_merge, and the HIP calls longer than 30 us inside it.
Usage: python tools/deshred_timeline.py <rocprofv3 output dir holding ht_*.csv>"""
import csv,sys
d=sys.argv[1]
k=list(csv.DictReader(open(d+'/ht_kernel_trace.csv')))
k.sort(key=lambda r:int(r['Start_Timestamp']))
a=list(csv.DictReader(open(d+'/ht_hip_api_trace.csv')))
a.sort(key=lambda r:int(r['Start_Timestamp']))
idx=[i for i,r in enumerate(k) if 'deserialize' in r['Kernel_Name']]
i0=idx[-1]
# end: first pipe_merge after i0
i1=next(i for i in range(i0,len(k)) if 'pipe_merge' in k[i]['Kernel_Name'])
t0=int(k[i0]['Start_Timestamp']); t1=int(k[i1]['End_Timestamp'])
prev=None; busy=0
for r in k[i0:i1+1]:
    s,e=int(r['Start_Timestamp']),int(r['End_Timestamp'])
    gap=(s-prev)/1e3 if prev else 0
    n=r['Kernel_Name'].replace('ag::(anonymous namespace)::','').replace('void ','')
    if gap>20 or (e-s)>300e3: print(f"{(s-t0)/1e3:9.1f} gap{gap:8.1f} dur{(e-s)/1e3:8.1f} q{r['Queue_Id']} {n[:60]}")
    prev=max(prev or 0,e)
print("span ms",(t1-t0)/1e6)
# long API calls in span
for r in a:
    s,e=int(r['Start_Timestamp']),int(r['End_Timestamp'])
    if s>=t0-2e6 and e<=t1+1e6 and e-s>30e3: print(f"API {(s-t0)/1e3:9.1f} {(e-s)/1e3:8.1f} {r['Function']}")

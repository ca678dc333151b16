"""Per-iteration kernel times and the gaps between them from a rocprofv3 kernel trace of bench.py
(one part): `python tools/iter_gaps.py <run_kernel_trace.csv>`.  Iterations are the kernels after
the last k_reset, each ending with k_finalize; the first five are skipped.  Used for the timing-marker
cost in DESIGN.md §6 (profiles/r06/coarse_timing/)."""
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# find iteration kernels: after the last k_reset
names=[r['Kernel_Name'] for r in rows]
idx=[i for i,n in enumerate(names) if 'k_reset' in n]
start=idx[-1]+1
its=[]; cur=[]
for r in rows[start:]:
    cur.append(r)
    if 'k_finalize' in r['Kernel_Name']:
        its.append(cur); cur=[]
print("iterations", len(its))
its=its[5:]
per=collections.defaultdict(list); span=[]; busy=[]
for it in its:
    t0=int(it[0]['Start_Timestamp']); t1=int(it[-1]['End_Timestamp'])
    span.append(t1-t0)
    b=0
    for r in it:
        d=int(r['End_Timestamp'])-int(r['Start_Timestamp']); b+=d
        per[r['Kernel_Name'].split('(')[0][:50]].append(d)
    busy.append(b)
# gap between iterations
gaps=[int(its[i+1][0]['Start_Timestamp'])-int(its[i][-1]['End_Timestamp']) for i in range(len(its)-1)]
import statistics as st
print("span us", st.median(span)/1e3, "busy us", st.median(busy)/1e3, "inter-iter gap us", st.median(gaps)/1e3)
for k,v in per.items(): print(f"  {k:50s} n={len(v)//len(its)} med={st.median(v)/1e3:.2f} us")
# intra gaps
ig=collections.defaultdict(list)
for it in its:
    for a,b in zip(it,it[1:]):
        ig[(a['Kernel_Name'][:25],b['Kernel_Name'][:25])].append(int(b['Start_Timestamp'])-int(a['End_Timestamp']))
for k,v in ig.items(): print("  gap",k,f"{st.median(v)/1e3:.2f}")

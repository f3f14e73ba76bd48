import numpy as np, sys
rows=[]; cur=[]
for line in open(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/trace.log'):
    if line.startswith('TRACE'):
        if cur: rows.append(cur)
        cur=[]
    elif line.startswith('B '):
        cur.append([int(x) for x in line.split()[1:]])
rows.append(cur)
a=np.array(rows[-1],dtype=np.int64)
b,t0,t1,t2,t3,t4,chunk,vis,t6,t7,t8,sw=a.T
t2=np.where(t2<0,t1,t2)
print("blocks",len(b),"total visits",vis.sum(),"chunk tot",chunk.sum())
def st(name,x):
    x=x[x>=0] if x.ndim else x
    print(f"{name:14s} med {np.median(x)/100:6.2f} p90 {np.percentile(x,90)/100:6.2f} max {x.max()/100:6.2f} us")
st("start",t0); st("end",t4)
st("scan",t1-t0); st("classify",t2-t1); st("visits",t3-t2); st("flush",t4-t3)
m=t6>=0
st("r0 start",(t6-t2)[m]); st("r0 visit",(t7-t6)[m]); st("r0 enqueue",(t8-t7)[m])
print("r0 sweeps dist", np.bincount(sw[m])[:40]); print("visits/block dist", np.bincount(vis)[:24])

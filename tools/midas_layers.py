"""Per-layer MiDaS v2.1-small kernel times against each layer's roofline bound (max of fp32 MFMA FLOPs at
the dense peak and the layer's input + output (+ residual) bytes at 8 TB/s), 32-frame batches, from a
rocprofv3 kernel trace of tools/bench_midas.py (tools/gpu_midas_splitk.sh).  Usage:
  python tools/midas_layers.py gpurun_out/<tag>/prof/midas_kernel_trace.csv
The layer list restates midas.hip Net::build() (shapes only); split-K finishing launches are
folded into their convolution."""
import csv, statistics as st
B=32; PEAK=157.3e12; HBM=8e12
layers=[]
def conv(t,cout,k,s,res=0):
    H,W,C=t; Ho,Wo=(H+s-1)//s,(W+s-1)//s
    fl=2*Ho*Wo*cout*C*k*k*B; by=(H*W*C+Ho*Wo*cout*(1+res))*4*B
    layers.append(('c%dx%d s%d'%(k,k,s),C,cout,Ho,fl,by)); return (Ho,Wo,cout)
def dw(t,k,s):
    H,W,C=t; Ho,Wo=(H+s-1)//s,(W+s-1)//s
    fl=2*Ho*Wo*C*k*k*B; by=(H*W*C+Ho*Wo*C)*4*B
    layers.append(('dw%d s%d'%(k,s),C,C,Ho,fl,by)); return (Ho,Wo,C)
def up(t):
    H,W,C=t; layers.append(('up',C,C,2*H,0,(H*W*C+4*H*W*C)*4*B)); return (2*H,2*W,C)
def ir(t,cout,k,s):
    cin=t[2]; x=conv(t,cin*6,1,1); x=dw(x,k,s); return conv(x,cout,1,1,res=1 if (s==1 and cin==cout) else 0)
def rcu(x,extra=0):
    c=x[2]; h=conv(x,c,3,1); return conv(h,c,3,1,res=1+extra)
def fusion(x0,x1,oc):
    o=rcu(x1,1) if x1 else x0; o=rcu(o); o=up(o); return conv(o,oc,1,1)
x=(256,256,3); x=conv(x,32,3,2); x=dw(x,3,1); x=conv(x,24,1,1)
skip=[]
for si,(c,k,s,n) in enumerate([(32,3,2,3),(48,5,2,3),(96,3,2,5),(136,5,1,5),(232,5,2,6),(384,3,1,1)]):
    for r in range(n): x=ir(x,c,k,s if r==0 else 1)
    if si in (0,1,3,5): skip.append(x)
rn=[conv(skip[0],64,3,1),conv(skip[1],128,3,1),conv(skip[2],256,3,1),conv(skip[3],512,3,1)]
p4=fusion(rn[3],None,256); p3=fusion(p4,rn[2],128); p2=fusion(p3,rn[1],64); p1=fusion(p2,rn[0],64)
o=conv(p1,32,3,1); o=up(o); o=conv(o,32,3,1); o=conv(o,1,1,1)
import sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows=[r for r in rows if 'midas' in r['Kernel_Name'] or 'wino3' in r['Kernel_Name']]
rows.sort(key=lambda r:int(r['Start_Timestamp']))
# fold split-K finishing launches into the preceding conv launch
merged=[]
for r in rows:
    if 'splitk' in r['Kernel_Name'] and merged:
        merged[-1]=dict(merged[-1]); merged[-1]['End_Timestamp']=r['End_Timestamp']; merged[-1]['Kernel_Name']=merged[-1]['Kernel_Name'].replace('(',' +sk(',1)
    else: merged.append(r)
rows=merged
n=len(layers); nb=len(rows)//n
print('launches',len(rows),'layers',n,'batches',nb)
tot=0; agg={}
for i,L in enumerate(layers):
    ds=[(int(rows[b*n+i]['End_Timestamp'])-int(rows[b*n+i]['Start_Timestamp']))/1e3 for b in range(1,nb)]
    kn=rows[n+i]['Kernel_Name'].split('(')[0].replace('vs::midas::','').replace('void vs::','')
    d=st.median(ds); bound=max(L[4]/PEAK,L[5]/HBM)*1e6; tot+=d
    key=L[0].split()[0][:4] if not L[0].startswith('c1x1') else 'c1x1'
    a=agg.setdefault(L[0]+' '+kn,[0,0]); a[0]+=d; a[1]+=bound
    print('%3d %-10s %-18s cin %4d cout %4d H %3d  %7.1f us  bound %6.1f  x%.1f'%(i,L[0],kn[:18],L[1],L[2],L[3],d,bound,d/bound))
print('total %.1f us'%tot)
for k,v in sorted(agg.items(),key=lambda kv:-kv[1][0]): print('%-40s %7.1f us bound %7.1f'%(k,v[0],v[1]))

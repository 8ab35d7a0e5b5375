"""Config-5 split-LSQR passes from rocprofv3 kernel traces: mean pass time alone vs beside the other slice's pass, per-kernel means, per-stream launch gaps.  python tools/pass_states.py DIR..."""
import csv,glob,sys,bisect
for d in sys.argv[1:]:
    path=sorted(glob.glob(d+'/**/*kernel_trace.csv',recursive=True))[0]
    ev=[]
    for r in csv.DictReader(open(path)):
        kn=r["Kernel_Name"]
        if "conic_fsplit_pass_kernel<4, 0>" in kn: k="P0"
        elif "conic_fsplit_pass_kernel<4, 1>" in kn: k="P1"
        elif "dpiU" in kn: k="U"
        elif "dpiV" in kn: k="V"
        else: continue
        ev.append((int(r["Start_Timestamp"]),int(r["End_Timestamp"]),k,r.get("Stream_Id",r.get("Queue_Id",""))))
    ev.sort()
    passes=[e for e in ev if e[2] in("P0","P1")]
    # for each pass: fraction of its duration overlapped by another pass
    starts=[e[0] for e in passes]
    alone=[];both=[]
    for i,(s,e,k,q) in enumerate(passes):
        ov=0
        for j in range(max(0,i-3),min(len(passes),i+4)):
            if j==i: continue
            s2,e2=passes[j][0],passes[j][1]
            ov+=max(0,min(e,e2)-max(s,s2))
        (both if ov>0.5*(e-s) else alone).append((e-s)/1000)
    import statistics as st
    print(d,'passes',len(passes),'alone n=%d mean %.1f us'%(len(alone),st.mean(alone) if alone else 0),'overlapped n=%d mean %.1f us'%(len(both),st.mean(both) if both else 0))
    for k in ("P0","P1","U","V"):
        ds=[(e-s)/1000 for s,e,kk,q in ev if kk==k]
        print('  ',k,'n',len(ds),'mean %.1f median %.1f'%(st.mean(ds),st.median(ds)))
    # gaps: per-stream gaps between consecutive launches
    byq={}
    for s,e,k,q in ev: byq.setdefault(q,[]).append((s,e,k))
    for q,l in byq.items():
        g=[(l[i+1][0]-l[i][1])/1000 for i in range(len(l)-1)]
        g=[x for x in g if x<50]
        print('  stream',q,'launches',len(l),'median gap %.2f us mean %.2f'%(st.median(g),st.mean(g)))

import sqlite3, numpy as np, collections, re, sys
c=sqlite3.connect(sys.argv[1])
rows=c.execute("select name, grid_x, duration, start from kernels order by start").fetchall()
inits=[s for n,gx,d,s in rows if 'k_pcg_init' in n]
t0=inits[1]; t1=max(s+d for n,gx,d,s in rows)
nit=len(inits)-1
sel=[r for r in rows if r[3]>=t0]
g=collections.defaultdict(list)
for n,gx,d,s in sel:
    m=re.search(r'(k_\w+)(<[^()]*>)?\(', n)
    key=((m.group(1)+(m.group(2) or '')) if m else n[:50], gx)
    g[key].append(d)
tot=sum(d for _,_,d,_ in sel)
print(f"window {(t1-t0)/1e6:.1f} ms for {nit} ADMM its -> {(t1-t0)/1e6/nit:.2f} ms/it; kernel sum {tot/1e6/nit:.2f} ms/it")
for (n,gx),ds in sorted(g.items(), key=lambda kv:-sum(kv[1]))[:28]:
    ds=np.array(ds)
    print(f"{ds.sum()/1e6/nit:7.2f} ms/it n/it={len(ds)/nit:6.1f} grid={gx:8d} avg={ds.mean()/1e3:7.1f}us {n}")

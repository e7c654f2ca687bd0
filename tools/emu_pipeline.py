"""CPU emulation of the GPU deflate pipeline (zs_k_prev, zs_k_match, zs_k_parse) for debugging parity."""
import sys
sys.path.insert(0,'/root/repo/tests')
import corpus, oracle
CFG = {4:(4,4,16,16),5:(8,16,32,32),6:(8,16,128,128),7:(8,32,128,256),8:(32,128,258,1024),9:(32,258,258,4096)}
MAXD = 32506
def stages(data, level):
    good, lazy, nice_cfg, chain = CFG[level]
    n = len(data)
    h = [((data[p]<<10)^(data[p+1]<<5)^data[p+2]) & 0x7fff if p+2 < n else -1 for p in range(n)]
    last = {}
    prevd = [0]*n
    for p in range(n):
        if p+2 < n:
            q = last.get(h[p]); d = p - q if q is not None else 0
            prevd[p] = d if d <= 32767 else 0
            last[h[p]] = p
    M = []
    for p in range(n):
        d0 = prevd[p] if p+2<n else 0; q0 = p-d0
        if not (d0 and q0 and d0 <= MAXD): M.append(None); continue
        look = n-p; maxc = min(look,258); nice = min(look, nice_cfg); limit = p-MAXD if p > MAXD else 0
        best, bq, cnt = 2, 0, 0; small=None; cur=q0
        while True:
            k=0
            while k < maxc and data[cur+k]==data[p+k]: k+=1
            if k > best:
                best, bq = k, cur
                if k >= nice: break
            cnt+=1
            if cnt == chain>>2: small=(best,bq)
            if cnt >= chain: break
            d = prevd[cur]
            if d == 0: break
            nx = cur-d
            if nx <= limit: break
            cur = nx
        if small is None: small=(best,bq)
        M.append(((best, p-bq if best>2 else 0), (small[0], p-small[1] if small[0]>2 else 0), d0==MAXD))
    enc = []
    for e in M:
        if e is None: enc.append((0, 0)); continue
        (b, d), (b2, d2), f = e
        enc.append(((b << 16) | d | (0x8000 if f else 0), (b2 << 16) | d2))
    syms=[]; p=0; ma=0; ml=2; ms=0; base=0
    while p < n:
        slid=False
        if p-base >= 65274 and min(n, base+65536)-p < 262: base+=32768; slid=True
        pl, pm = ml, ms; ml=2
        e = M[p]
        if e is not None and pl < lazy and not (slid and e[2]):
            L, D = e[1] if pl >= good else e[0]
            if L > pl:
                ml=L; ms=p-D
                if L==3 and D>4096: ml=2
        if pl>=3 and ml<=pl:
            syms.append(0x80000000 | ((pl-3) << 16) | (p-1-pm)); p += pl-1; ma=0; ml=2
        elif ma:
            syms.append(data[p-1]); p+=1
        else:
            ma=1; p+=1
    if ma: syms.append(data[p-1])
    return prevd, enc, syms

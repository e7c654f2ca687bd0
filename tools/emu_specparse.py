"""CPU emulation of the segment-parallel speculative parse (deflate_parse.hip)
checked against the serial lazy parse, with small segments to stress splices.
usage: python tools/emu_specparse.py"""
import sys
sys.path.insert(0, '/root/repo/tools')
sys.path.insert(0, '/root/repo/tests')
import corpus
from emu_pipeline import stages, CFG

NONE = None


def step(st, e, lit, n, good, lazy):
    p, ma, pl, pm = st
    ml, ms = 2, pm
    ex, ey = e
    nil = (ex & 0x8000) and p >= 65274 and (p - 65274) % 32768 == 0 and n - p < 262
    if (ex >> 16) and pl < lazy and not nil:
        u = ey if pl >= good else ex
        L, D = u >> 16, u & 0x7fff
        if L > pl:
            ml, ms = L, p - D
            if L == 3 and D > 4096:
                ml = 2
    if pl >= 3 and ml <= pl:
        return (p + pl - 1, 0, 2, ms), 0x80000000 | ((pl - 3) << 16) | (p - 1 - pm)
    if ma:
        return (p + 1, 1, ml, ms), lit
    return (p + 1, 1, ml, ms), NONE


def specparse(data, enc, level, SEG):
    good, lazy, _, _ = CFG[level]
    n = len(data)
    lit = lambda p: data[p - 1] if p > 0 else 0
    nseg = (n + SEG - 1) // SEG
    spec = []
    for k in range(nseg):
        a, b = k * SEG, min(n, k * SEG + SEG)
        st = (a, 0, 2, 0); out = []; sync = {}
        while st[0] < b:
            if st[2] == 2:
                sync[(st[0], st[1])] = len(out)
            st, v = step(st, enc[st[0]], lit(st[0]), n, good, lazy)
            if v is not NONE:
                out.append(v)
        if b == n and st[1]:
            out.append(data[n - 1])
        spec.append((st, out, sync))
    t = (0, 0, 2, 0); res = []; catch = 0; nosync = 0
    for k in range(nseg):
        a, b = k * SEG, min(n, k * SEG + SEG)
        st_end, out, sync = spec[k]
        frm = None
        while t[0] < b:
            if t[2] == 2 and (t[0], t[1]) in sync:
                frm = sync[(t[0], t[1])]; break
            t, v = step(t, enc[t[0]], lit(t[0]), n, good, lazy)
            catch += 1
            if v is not NONE:
                res.append(v)
        if frm is not None:
            res.extend(out[frm:]); t = st_end
        else:
            nosync += 1
            if b == n and t[1]:
                res.append(data[n - 1])
    return res, catch, nosync


if __name__ == '__main__':
    cases = [('text', 3, 70000), ('mixed', 5, 40000), ('text', 9, 65536 + 100), ('rand', 1, 5000),
             ('text', 11, 98305), ('zeros', 0, 70000)]
    for kind, seed, n in cases:
        data = bytes(n) if kind == 'zeros' else getattr(corpus, kind)(seed, n)
        for level in (6, 9, 4):
            _, enc, syms = stages(data, level)
            for SEG in (64, 1024):
                got, catch, nosync = specparse(data, enc, level, SEG)
                ok = got == syms
                print(kind, seed, n, 'L%d' % level, 'SEG', SEG, 'OK' if ok else 'MISMATCH', 'catch-up steps', catch,
                      'no-sync segs', nosync, flush=True)
                if not ok:
                    sys.exit(1)

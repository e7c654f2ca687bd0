"""CPU model of the two-kernel lazy parse (zs_k_parse_a / zs_k_parse_b,
deflate_parse2.hip), mirroring the kernels' control flow lane by lane, checked
against the serial lazy parse (tools/emu_pipeline.py) for symbols.
usage: python tools/emu_parse_split.py [SEG LANES]"""
import sys

sys.path.insert(0, '/root/repo/tools')
sys.path.insert(0, '/root/repo/tests')
import corpus  # noqa: E402
from emu_pipeline import stages, CFG  # noqa: E402
from emu_specparse import step as step_t  # noqa: E402

NONE = None


def clean_eq(a, b):
    return a[2] == 2 and b[2] == 2 and a[0] == b[0] and a[1] == b[1]


def split_parse(data, enc, level, SEG=64, LANES=64):
    good, lazy, _, _ = CFG[level]
    n = len(data)
    RANGE = SEG * LANES
    lit = lambda p: data[p - 1] if p > 0 else 0  # noqa: E731

    def step(st):
        st2, v = step_t(st, enc[st[0]], lit(st[0]), n, good, lazy)
        return st2, v

    nr = (n + RANGE - 1) // RANGE
    recs = []
    fallbacks = 0
    # ---- kernel A
    for r in range(nr):
        r0 = r * RANGE
        rend = min(n, r0 + RANGE)
        lanes = []
        for j in range(LANES):
            a = r0 + j * SEG
            b = min(n, a + SEG)
            act = a < n
            E = (a, 0, 2, 0)
            nspec = 0
            if act:
                while E[0] < b:
                    E, v = step(E)
                    nspec += v is not NONE
                if b == n and E[1]:
                    nspec += 1
            sy = sma = sk = nt = 0
            ok = True
            a1 = a + SEG
            cap = min(n, a1 + 3 * SEG)
            if act and j < LANES - 1 and a1 < rend:
                ok = False
                T, S = E, (a1, 0, 2, 0)
                while True:
                    if clean_eq(T, S) or (T[0] >= n and S[0] >= n and T[1] == S[1]):
                        ok = True
                        break
                    if S[0] >= cap or T[0] >= cap:
                        break
                    adv_t, adv_s = T[0] <= S[0], S[0] <= T[0]
                    if adv_t:
                        T, v = step(T)
                        nt += v is not NONE
                    if adv_s:
                        S, v = step(S)
                        sk += v is not NONE
                sy, sma = S[0], S[1]
            lanes.append(dict(a=a, b=b, act=act, E=E, nspec=nspec, sy=sy, sma=sma, sk=sk, nt=nt, ok=ok))
        rec = dict(lane=[None] * LANES)
        # Entry of the true path into each lane's path P_k (the parse from a_k,
        # continued by its T_k): position Y and how many of P_k's symbols precede
        # it.  If Y lies past P_k's own meeting y_k, P_k has already merged into
        # P_{k+1}: lane k contributes nothing and the entry moves on.
        Y, skip = r0, 0
        order_ok = True
        for j, L in enumerate(lanes):
            if not L['act']:
                break
            merges = j < LANES - 1 and L['a'] + SEG < rend
            out = L['nspec'] + L['nt']
            yk = L['sy'] if merges else L['E'][0]
            if Y <= yk:
                L['skip'], L['contrib'] = skip, True
                if merges:
                    Y, skip = L['sy'], L['sk']
            else:
                L['skip'], L['contrib'] = 0, False
                if not merges:
                    order_ok = False  # the true path joins past the range's end
                else:
                    skip = L['sk'] + (skip - out)
        if all(L['ok'] for L in lanes) and order_ok:
            run = []
            for j, L in enumerate(lanes):
                if not L['act']:
                    continue
                skip = L['skip'] if L['contrib'] else 1 << 30
                st = (L['a'], 0, 2, 0)
                i = 0
                while st[0] < L['b']:
                    st, v = step(st)
                    if v is not NONE:
                        if i >= skip:
                            run.append(v)
                        i += 1
                fin = L['b'] == n and st[1]
                if fin:
                    if i >= skip:
                        run.append(data[n - 1])
                    i += 1
                if L['nt']:
                    T = st
                    while not (T[2] == 2 and T[0] == L['sy'] and T[1] == L['sma']):
                        T, v = step(T)
                        if v is not NONE:
                            if i >= skip:
                                run.append(v)
                            i += 1
                if L['b'] >= rend:
                    rec.update(run=run, serial=False, fin=fin, E=st)
        else:
            fallbacks += 1
            st = (r0, 0, 2, 0)
            run = []
            while st[0] < rend:
                st, v = step(st)
                if v is not NONE:
                    run.append(v)
            fin = rend == n and st[1]
            if fin:
                run.append(data[n - 1])
            rec.update(run=run, serial=True, fin=fin, E=st)
            rec['lane'][0] = (r0, 0, 0)
        recs.append(rec)

    # ---- kernel B
    def join(T, r):
        r0 = r * RANGE
        rend = min(n, r0 + RANGE)
        fix = []
        S = (r0, 0, 2, 0)  # the range's run is the parse from r0 (fresh), continued
        sk = 0
        while True:
            if clean_eq(T, S):
                return sk, fix, False, T
            if T[0] >= rend:
                break
            adv_t = T[0] <= S[0]
            adv_s = S[0] <= T[0]
            if adv_t:
                T, v = step(T)
                if v is not NONE:
                    fix.append(v)
            if adv_s:
                S, v = step(S)
                sk += v is not NONE
        fin = False
        if rend == n and T[1]:
            fix.append(data[n - 1])
            fin = True
        return None, fix, fin, T

    cut = [0] * nr
    fixes = [[] for _ in range(nr)]
    for r in range(1, nr):  # parallel attempt
        c, fx, fin, _ = join(recs[r - 1]['E'], r)
        cut[r], fixes[r] = c, fx
    if any(c is None for c in cut[1:]):
        r = 1
        while r < nr and cut[r] is not None:
            r += 1
        T = recs[r - 1]['E']
        while r < nr:
            c, fx, fin, T2 = join(T, r)
            cut[r], fixes[r] = c, fx
            T = recs[r]['E'] if c is not None else T2
            r += 1
    out = []
    for r in range(nr):
        out.extend(fixes[r])
        if cut[r] is not None:
            out.extend(recs[r]['run'][cut[r]:])
    return out, fallbacks


if __name__ == '__main__':
    SEG = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    LANES = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    cases = [('text', 3, 777), ('text', 3, 70000), ('mixed', 5, 40000), ('text', 9, 65536 + 100),
             ('rand', 1, 5000), ('zeros', 0, 20000), ('text', 11, 9000)]
    for kind, seed, n in cases:
        data = bytes(n) if kind == 'zeros' else getattr(corpus, kind)(seed, n)
        for level in (4, 6, 9):
            _, enc, syms = stages(data, level)
            got, fb = split_parse(data, enc, level, SEG, LANES)
            ok = got == syms
            print(kind, seed, n, 'L%d' % level, 'OK' if ok else 'MISMATCH', 'fallback ranges', fb, flush=True)
            if not ok:
                i = next((i for i in range(min(len(got), len(syms))) if got[i] != syms[i]), min(len(got), len(syms)))
                print('  first difference at symbol', i, 'got', got[i:i + 3], 'want', syms[i:i + 3], len(got),
                      len(syms))
                sys.exit(1)

#!/usr/bin/env python3
"""LDS bank-conflict model of the column kernel's twiddle-table reads (development tool).

Re-implements rs_mono.hip's compile-time plan (seg_map / layers / Plan) and LdsTabs::get's
slot arithmetic, enumerates every ds_read_b128 of a table (per layer, wave, register pair)
and counts LDS cycles per lane group ({0-3,12-15,20-27}, ... per the MI355X guide's LDS
table) for candidate slot maps: the 20-word stride, paddings, and XOR swizzles of the slot
or of the group index within a layer.  Run: python3 tools/lds_bank_model.py
"""
# Python model of rs_mono.hip's compile-time plan and LdsTabs::get slot reads: LDS bank
# conflicts of the staged kernel's twiddle-table reads for candidate slot address maps.
import itertools
KXPOSE, KLAYER, KREMAP = 2, 1, 3
def seg_map(L, LR, lo, order):
    IW = LR + 6
    pri = []
    for x in order:
        if x < lo or x >= lo + IW or x in pri: continue
        pri.append(x)
    for x in range(lo, lo + IW):
        if x not in pri: pri.append(x)
    pref = [5, 4, 0, 1, 3, 2]
    m = {'reg': [pri[s] if s < LR else -1 for s in range(3)], 'lane': [0]*6, 'wave': []}
    for j in range(6): m['lane'][pref[j]] = pri[LR + j]
    m['wave'] = [x for x in range(L) if x < lo or x >= lo + IW] + [-1]*4
    m['wave'] = m['wave'][:4]
    return m
def cp(m): return {'reg': list(m['reg']), 'lane': list(m['lane']), 'wave': list(m['wave'])}
def layers(ops, maps, m, LR, bits):
    for t, x in enumerate(bits):
        rs = m['reg'].index(x) if x in m['reg'][:LR] else -1
        if rs < 0:
            j = m['lane'].index(x)
            far = -1
            for q in range(LR):
                u = next((tt for tt in range(t + 1, len(bits)) if bits[tt] == m['reg'][q]), 1 << 20)
                if u > far: far, rs = u, q
            m['reg'][rs], m['lane'][j] = m['lane'][j], m['reg'][rs]
            ops.append((KXPOSE, x, rs, j)); maps.append(cp(m))
        ops.append((KLAYER, x, rs, 0)); maps.append(cp(m))
def plan(L, LR, SPLIT):
    IW = LR + 6; WB = L - IW - (1 if SPLIT else 0); TOP = L - 1 if SPLIT else L
    # ifft
    ops, maps = [], []
    order = list(range(IW))
    m = seg_map(L, LR, 0, order); maps.append(cp(m))
    layers(ops, maps, m, LR, list(range(IW)))
    order = list(range(IW, TOP)) + list(range(TOP - 1, WB - 1, -1))
    m = seg_map(L, LR, WB, order); ops.append((KREMAP, -1, 0, 0)); maps.append(cp(m))
    layers(ops, maps, m, LR, list(range(IW, TOP)))
    ifft = (ops, maps)
    ops2, maps2 = [], [cp(maps[-1])]
    m = cp(maps[-1])
    layers(ops2, maps2, m, LR, list(range(TOP - 1, WB - 1, -1)))
    if WB > 0:
        m = seg_map(L, LR, 0, list(range(WB - 1, -1, -1))); ops2.append((KREMAP, -1, 0, 0)); maps2.append(cp(m))
        layers(ops2, maps2, m, LR, list(range(WB - 1, -1, -1)))
    return ifft, (ops2, maps2)
def lane_rows(m, lane, wave):
    r = 0
    for j in range(6): r |= ((lane >> j) & 1) << m['lane'][j]
    for k in range(4):
        if m['wave'][k] >= 0: r |= ((wave >> k) & 1) << m['wave'][k]
    return r
def reg_rows(m, LR, i):
    return sum(((i >> s) & 1) << m['reg'][s] for s in range(LR))
GROUPS = [list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
GROUPS += [[g+32 for g in G] for G in GROUPS]
def reads(L, LR, SPLIT, B0, dec):
    """(phase, region, [per wave: per register-pair: lane -> slot]) for every table read."""
    IW = LR + 6; W = 1 << IW; n = 1 << L; WB = L - IW - (1 if SPLIT else 0); TOP = L - 1 if SPLIT else L
    kShI = (n >> IW) - 1 if WB > 0 else 0
    nw = 1 << (L - LR - 6)
    out = []
    for FFT, (ops, maps) in enumerate(plan(L, LR, SPLIT)):
        ri = next((i for i, o in enumerate(ops) if o[0] == KREMAP), len(ops))
        for I, o in enumerate(ops):
            if o[0] != KLAYER: continue
            x, rs = o[1], o[2]
            ph = (3 if I >= ri else 4) if FFT else (1 if I < ri else 2)
            if ri == len(ops): ph = 3 if FFT else 1
            m = maps[I]
            for wave in range(nw):
                for i in range(1 << LR):
                    if (i >> rs) & 1: continue
                    slots = []
                    for lane in range(64):
                        row = lane_rows(m, lane, wave) | reg_rows(m, LR, i)
                        if ph in (1, 3):
                            if B0 and x == 0: slot = (row & (W - 1)) >> 1; reg = 'priv'
                            else: slot = (W >> B0) - (W >> x) + ((row & (W - 1)) >> (x + 1)); reg = 'priv'
                        elif ph == 2: slot = (n >> IW) - (n >> x) + (row >> (x + 1)); reg = 'sh'
                        else: slot = kShI + (n >> WB) - (n >> x) + (row >> (x + 1)); reg = 'sh'
                        slots.append(slot)
                    out.append((ph, reg, slots))
    return out
def cycles(slot_reads, addr):
    tot = 0; ideal = 0
    for ph, reg, slots in slot_reads:
        for G in GROUPS:
            quads = {}
            for l in G:
                a = addr(slots[l])  # word address of piece 0
                quads.setdefault((a // 4) % 16, set()).add(a)
            tot += max(len(v) for v in quads.values()); ideal += 1
    return tot, ideal
import sys
cands = {
  'stride20': lambda s: 20 * s,
  'pad4per16': lambda s: 20 * s + 4 * (s >> 4),
  'pad4per8': lambda s: 20 * s + 4 * (s >> 3),
  'pad4per4': lambda s: 20 * s + 4 * (s >> 2),
  'xor4': lambda s: 20 * (s ^ ((s >> 4) & 15)),
  'xor2': lambda s: 20 * (s ^ ((s >> 2) & 3)),
  'xor3': lambda s: 20 * (s ^ ((s >> 3) & 7)),
  'stride24': lambda s: 24 * s,
  'stride28': lambda s: 28 * s,
}
for (L, LR, SPLIT, B0, dec, name) in [(10, 1, False, 0, False, 'encode L10'), (11, 1, True, 1, True, 'decode L11 split'), (9,1,False,0,False,'L9')]:
    rd = reads(L, LR, SPLIT, B0, dec)
    print(name, len(rd), 'reads')
    for cn, f in cands.items():
        for ph in (1, 2, 3, 4):
            pass
        t, i = cycles(rd, f)
        byph = {}
        for ph in (1,2,3,4):
            sub = [r for r in rd if r[0] == ph]
            if sub: byph[ph] = round(cycles(sub, f)[0] / cycles(sub, f)[1], 2)
        print(f"  {cn:10s} conflict factor {t/i:.3f}  by phase {byph}")

print("---- per-layer search")
def reads_x(L, LR, SPLIT, B0):
    IW = LR + 6; W = 1 << IW; n = 1 << L; WB = L - IW - (1 if SPLIT else 0)
    kShI = (n >> IW) - 1 if WB > 0 else 0
    nw = 1 << (L - LR - 6)
    out = []
    for FFT, (ops, maps) in enumerate(plan(L, LR, SPLIT)):
        ri = next((i for i, o in enumerate(ops) if o[0] == KREMAP), len(ops))
        for I, o in enumerate(ops):
            if o[0] != KLAYER: continue
            x, rs = o[1], o[2]
            ph = (3 if I >= ri else 4) if FFT else (1 if I < ri else 2)
            m = maps[I]
            for wave in range(nw):
                for i in range(1 << LR):
                    if (i >> rs) & 1: continue
                    gs = []
                    for lane in range(64):
                        row = lane_rows(m, lane, wave) | reg_rows(m, LR, i)
                        if ph in (1, 3): g = (row & (W - 1)) >> (x + 1); key = ('priv', x)
                        else: g = row >> (x + 1); key = ('sh', x, ph)
                        gs.append(g)
                    out.append((key, gs))
    return out
def cyc(gs_list, f):
    t = 0
    for gs in gs_list:
        for G in GROUPS:
            q = {}
            for l in G:
                a = f(gs[l]); q.setdefault((a // 4) % 16, set()).add(a)
            t += max(len(v) for v in q.values())
    return t
fams = {'id': lambda g: g}
for a in range(1, 7):
    for mb in (1, 3, 7, 15):
        fams[f'x{a}_{mb}'] = (lambda a, mb: (lambda g: g ^ ((g >> a) & mb)))(a, mb)
for (L, LR, SPLIT, B0, name) in [(10, 1, False, 0, 'encode L10'), (11, 1, True, 1, 'decode L11 split')]:
    rx = reads_x(L, LR, SPLIT, B0)
    keys = sorted(set(k for k, _ in rx), key=str)
    tot_id = tot_best = ideal = 0
    for k in keys:
        gl = [gs for kk, gs in rx if kk == k]
        base = cyc(gl, lambda g: 20 * g)
        best = min(((cyc(gl, (lambda f: (lambda g: 20 * f(g)))(f)), fn) for fn, f in fams.items()), key=lambda t: t[0])
        tot_id += base; tot_best += best[0]; ideal += len(gl) * 4
        print(f"  {name} {str(k):18s} reads {len(gl):4d} stride20 {base/(len(gl)*4):.2f} best {best[0]/(len(gl)*4):.2f} {best[1]}")
    print(name, 'total', tot_id / ideal, '->', tot_best / ideal)

print("---- global sigma")
for (L, LR, SPLIT, B0, name) in [(10, 1, False, 0, 'encode L10'), (11, 1, True, 1, 'decode L11 split'), (9, 1, False, 0, 'L9'), (8, 1, False, 0, 'L8'), (11, 1, False, 1, 'L11 nosplit'), (9, 1, True, 0, 'L9 split'), (10, 1, True, 0, 'L10 split')]:
    rx = reads_x(L, LR, SPLIT, B0)
    ideal = sum(4 for _ in rx)
    for fn in ('id', 'x1_15', 'x1_7', 'x1_3'):
        f = fams[fn]
        t = sum(cyc([gs], (lambda f: (lambda g: 20 * f(g)))(f)) for _, gs in rx)
        print(f"  {name:18s} {fn:6s} {t/ideal:.3f}")

"""Independent pure-Python restatement of the reference decoders, for SMALL
cases only: a second, literal transcription of src/qkd_ldpc_algorithm.cpp
(nested lists, the reference's loop order, math.tanh/math.atanh from the C
library) used to cross-check the C oracle.  Test infrastructure only."""
import math
import sys

DBL_MAX = sys.float_info.max


def _clip(mat, thr):
    for row in mat:
        for k, v in enumerate(row):
            if v > thr:
                row[k] = thr
            elif v < -thr:
                row[k] = -thr


def _tanh_lin(x):
    a = abs(x)
    if a < 0.5: r = 0.9242 * a
    elif a < 0.9: r = 0.6355 * a + 0.1444
    elif a < 1.2: r = 0.3912 * a + 0.3642
    elif a < 1.75: r = 0.1958 * a + 0.5986
    elif a < 2.5: r = 0.0603 * a + 0.8358
    elif a < 3.5: r = 0.0115 * a + 0.9577
    elif a < 8: r = 0.0004 * a + 0.9967
    else: r = 1.0
    return -r if x < 0. else r


def _atanh_lin(x):
    a = abs(x)
    if a < 0.7: r = 1.196 * a - 0.0323
    elif a < 0.9: r = 2.9187 * a - 1.214
    elif a < 0.999: r = 10.8717 * a - 8.3717
    else: r = 2510.9 * a - 2505.9
    return -r if x < 0. else r


def _atanh(x):
    try:
        return math.atanh(x)
    except ValueError:  # C atanh: +-1 -> +-inf, |x|>1 -> NaN
        if x == 1.0: return math.inf
        if x == -1.0: return -math.inf
        return math.nan


def decode(check_nodes, bit_nodes, alg, llr, syndrome, max_it, thr_on, thr, primary=0.0, secondary=0.0):
    """-> (out bits list, iterations, syndromes_match, total_bit_llr list)"""
    n, m = len(bit_nodes), len(check_nodes)
    b2c = [[llr[i] for i in check_nodes[j]] for j in range(m)]
    c2b = [[0.0] * len(bit_nodes[i]) for i in range(n)]
    total = [0.0] * n
    adaptive = alg in (4, 5)
    out = [(1 if llr[i] <= 0 else 0) for i in range(n)] if adaptive else [0] * n
    for it in range(max_it):
        cpos = [0] * n
        eq_all = True
        for j in range(m):
            if alg in (0, 1):
                rp = -1. if syndrome[j] else 1.
                for k in range(len(check_nodes[j])):
                    x = b2c[j][k] / 2.
                    b2c[j][k] = math.tanh(x) if alg == 0 else _tanh_lin(x)
                    rp *= b2c[j][k]
                for k, i in enumerate(check_nodes[j]):
                    p = rp / b2c[j][k] if b2c[j][k] != 0 else (math.copysign(math.inf, rp) * math.copysign(1, b2c[j][k]) if rp != 0 else math.nan)
                    c2b[i][cpos[i]] = 2. * (_atanh(p) if alg == 0 else _atanh_lin(p))
                    cpos[i] += 1
            else:
                sp = -1. if syndrome[j] else 1.
                neg = 0
                m1 = m2 = DBL_MAX
                for v in b2c[j]:
                    if v < 0: neg += 1
                    a = abs(v)
                    if a < m1: m2, m1 = m1, a
                    elif a < m2: m2 = a
                sp *= 1. if neg % 2 == 0 else -1.
                fac = primary
                if adaptive:
                    d = 0
                    for i in check_nodes[j]: d ^= out[i]
                    if d != syndrome[j]:
                        fac = secondary
                        eq_all = False
                for k, i in enumerate(check_nodes[j]):
                    v = b2c[j][k]
                    prod = sp * (1. if v > 0 else -1.)
                    sel = m2 if abs(v) == m1 else m1
                    if alg in (2, 4):
                        c2b[i][cpos[i]] = fac * prod * sel
                    else:
                        diff = sel - fac
                        c2b[i][cpos[i]] = prod * (0. if diff < 0. else diff)
                    cpos[i] += 1
        if adaptive and eq_all:
            return out, it + 1, True, total
        if thr_on: _clip(c2b, thr)
        for i in range(n):
            acc = llr[i]
            for v in c2b[i]: acc = acc + v
            total[i] = acc
            out[i] = 1 if acc <= 0 else 0
        if not adaptive:
            ok = True
            for j in range(m):
                s = 0
                for i in check_nodes[j]: s ^= out[i]
                if s != syndrome[j]:
                    ok = False
                    break
            if ok:
                return out, it + 1, True, total
        bpos = [0] * m
        for i in range(n):
            for k, j in enumerate(bit_nodes[i]):
                b2c[j][bpos[j]] = total[i] - c2b[i][k]
                bpos[j] += 1
        if thr_on: _clip(b2c, thr)
    return out, max_it, False, total

"""The arithmetic of MSP_REDUCE_SEQ's exact parallel engine (csrc/msplit_seq.hip), restated in Python integers.

The device engine rebuilds a sequential sum s = fl(s + p_i) (the reference's f2cblaslapack ddot order, oracle
ORC_REDUCE_SEQ) from "transducers": while s stays in one binade [2^e, 2^(e+1)) of one sign it is M * 2^(e-52) with
M an integer in [2^52, 2^53), and each term adds floor(p / u) plus a rounding bit to M (a tie rounds to even M, so
the map depends on M's parity).  A run of terms is, per input parity, an offset d with the lowest exact sum lo and
the highest result hi; runs compose associatively and apply to an actual s only when M + lo >= 2^52 and
M + hi < 2^53.  This file restates decomp / the lane run / tr_comb / tr_apply exactly as the kernel computes them
and checks, on the CPU and against the f64 sequential sum itself, that (a) any composition order of the runs
gives the same map, (b) a walk that applies whatever is valid and adds the rest term by term reproduces the
sequential sum bit for bit on adversarial inputs (dense ties at both parities, exact powers of two, returns to
+0.0, subnormals, huge ranges, +-inf), whatever the guessed binades were.  The GPU kernels themselves are checked
against the oracle in tests/test_gpu_seq_engine.py.
"""
import math
import struct

import numpy as np
import pytest

M0, M1, BIG, LIM = 1 << 52, 1 << 53, 1 << 60, 1 << 56
FRAC = (1 << 52) - 1


def bits(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def fromb(b):
    return struct.unpack("<d", struct.pack("<Q", b))[0]


def decomp(p, e, sneg):
    """(q, class) of p / 2^(e-52) (sign-flipped for a negative state), or None (non-finite or |p| >= 2^(e+1))."""
    b = bits(p)
    E = (b >> 52) & 0x7FF
    if E == 0x7FF:
        return None
    m = b & FRAC
    if E:
        m |= 1 << 52
    else:
        E = 1
    if m == 0:
        return 0, 0
    sh = E - 1023 - e
    if sh > 0:
        return None
    neg = (b >> 63) != sneg
    k = min(-sh, 63)
    if k == 0:
        return (-m if neg else m), 0
    qq, rr, half = m >> k, m & ((1 << k) - 1), 1 << (k - 1)
    if not neg:
        return qq, (2 if rr > half else (1 if rr == half else 0))
    if rr == 0:
        return -qq, 0
    return -qq - 1, (2 if rr < half else (1 if rr == half else 0))


def ident():
    return dict(d=[0, 0], lo=[BIG, BIG], hi=[-BIG, -BIG], e=0, neg=0, bad=False, zero=True, nzero=True)


def run(ps, e, sneg, gok, dec=decomp):
    """The lane run of k_seqx_trans: terms decomposed once, parity 0's track, parity 1's only if a tie occurs."""
    t = ident()
    qc = []
    for p in ps:
        b = bits(p)
        if (b << 1) & ((1 << 64) - 1) == 0:
            if not (b >> 63):
                t["nzero"] = False
            qc.append(None)
            continue
        if t["zero"]:
            t.update(zero=False, nzero=False, neg=sneg, e=e)
        r = dec(p, e, sneg) if gok else None
        if r is None:
            t["bad"] = True
            r = (0, 0)
        qc.append((int(r[0]), r[1]))
    if t["zero"]:
        return t
    tie = False
    for pi in (0, 1):
        if pi == 1 and not tie:
            t["d"][1], t["lo"][1], t["hi"][1] = t["d"][0], t["lo"][0], t["hi"][0]
            break
        for r in qc:
            if r is None:
                continue
            q, c = r
            t["lo"][pi] = min(t["lo"][pi], t["d"][pi] + q)
            t["d"][pi] += q + (1 if c == 2 else 0) + (((pi + t["d"][pi] + q) & 1) if c == 1 else 0)
            t["hi"][pi] = max(t["hi"][pi], t["d"][pi])
            tie |= c == 1
    if abs(t["d"][0]) > LIM or abs(t["d"][1]) > LIM:
        t["bad"] = True
        t["d"] = [0, 0]
    return t


def comb(a, b):
    if a["zero"]:
        r = {k: (list(v) if isinstance(v, list) else v) for k, v in b.items()}
        if not a["nzero"]:
            r["nzero"] = False
        return r
    if b["zero"]:
        return a
    r = dict(e=a["e"], neg=a["neg"], zero=False, nzero=False, d=[0, 0], lo=[0, 0], hi=[0, 0],
             bad=a["bad"] or b["bad"] or a["e"] != b["e"] or a["neg"] != b["neg"])
    for pi in (0, 1):
        ad = a["d"][pi]
        p2 = (pi + ad) & 1
        r["d"][pi] = ad + b["d"][p2]
        r["lo"][pi] = max(-BIG, min(BIG, min(a["lo"][pi], ad + b["lo"][p2])))
        r["hi"][pi] = max(-BIG, min(BIG, max(a["hi"][pi], ad + b["hi"][p2])))
    if abs(r["d"][0]) > LIM or abs(r["d"][1]) > LIM:
        r["bad"] = True
        r["d"] = [0, 0]
    return r


def apply(t, s):
    if t["zero"]:
        if s == 0.0:
            return -0.0 if (math.copysign(1.0, s) < 0 and t["nzero"]) else 0.0
        return s
    if t["bad"]:
        return None
    b = bits(s)
    E = (b >> 52) & 0x7FF
    if E in (0, 0x7FF) or E - 1023 != t["e"] or (b >> 63) != t["neg"]:
        return None
    M = (b & FRAC) | (1 << 52)
    pi = M & 1
    if M + t["lo"][pi] < M0 or M + t["hi"][pi] >= M1:
        return None
    return fromb((b & ~FRAC & ((1 << 64) - 1)) | (M + t["d"][pi] - M0))


def guess(G):
    b = bits(G)
    E = (b >> 52) & 0x7FF
    return E not in (0, 0x7FF), E - 1023, b >> 63


def seqsum(ps, s=0.0):
    for p in ps:
        s = s + p
    return s


def engine(ps, sub=16, per=4, jitter=1e-9, seed=0, dec=None, s0=0.0):
    """Sub-segment transducers built from lane runs of `per` terms in the binade of a jittered guess, applied where
    valid; the rest term by term with the f64 add (the walk's serial sub-segments).  s0: the exact state the sum
    starts from (mspi_seq_chain's acc_in: the previous row block's result; the guesses start there too)."""
    rng = np.random.default_rng(seed)
    pre = s0 + np.concatenate([[0.0], np.cumsum(ps)])
    s, i, n, fast = s0, 0, len(ps), 0
    while i < n:
        j = min(n, i + sub)
        gok, e, sn = guess(float(pre[i]) * (1.0 + jitter * rng.uniform(-1, 1)))
        lanes = [run(ps[k:min(k + per, j)], e, sn, gok, dec or decomp) for k in range(i, j, per)]
        t = lanes[0]
        for u in lanes[1:]:
            t = comb(t, u)
        r = apply(t, s)
        if r is not None:
            s, fast = r, fast + 1
        else:
            s = seqsum(ps[i:j], s)
        i = j
    return s, fast


def _cases():
    rng = np.random.default_rng(20251121)
    tie_terms = [-3.0, -1.0, 1.0, 3.0, 5.0, -5.0, 0.5, -0.5, 2.0]
    return {
        "walk": rng.standard_normal(6000) * rng.standard_normal(6000),
        "ties_even": np.concatenate([[2.0 ** 53], rng.choice(tie_terms, 3000)]),
        "ties_odd": np.concatenate([[2.0 ** 52 + 1], rng.choice(tie_terms, 3000)]),
        "quarter": np.full(6000, 0.25),
        "cancel": np.repeat(rng.uniform(-1, 1, 1500), 2) * np.tile([1.0, -1.0], 1500),
        "small_on_large": np.concatenate([[1e16], np.full(3000, 1e-3)]),
        "range": np.sign(rng.standard_normal(4000)) * 10.0 ** rng.uniform(-150, 150, 4000),
        "drift": rng.uniform(0.5, 1, 4000) * rng.uniform(-0.2, 1, 4000),
        "subnormal": rng.uniform(-1, 1, 1500) * 1e-160 * rng.uniform(0, 1, 1500) * 1e-160,
        "neg_zero": np.full(100, -0.0),
        "inf": np.concatenate([rng.uniform(-1, 1, 500), [np.inf], rng.uniform(-1, 1, 500)]),
        "overflow": np.full(300, 1e307),
    }


CASES = _cases()


@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("jitter", [0.0, 1e-9, 0.3])
@pytest.mark.parametrize("dec", ["int", "f64"])
def test_engine_walk_is_the_sequential_sum(name, jitter, dec):
    ps = [float(v) for v in CASES[name]]
    ref = seqsum(ps)
    got, fast = engine(ps, jitter=jitter, dec=decomp if dec == "int" else globals()["decomp_f"])
    assert bits(got) == bits(ref), (got, ref)


@pytest.mark.parametrize("name", ["walk", "ties_even", "ties_odd", "cancel", "drift", "small_on_large", "range"])
def test_engine_chained_pieces_are_the_sequential_sum(name):
    """mspi_seq_chain: a sum cut into pieces (the LSQR's row blocks, empty ones included), each piece walked from
    the previous piece's exact result, is the one sequential sum."""
    ps = [float(v) for v in CASES[name]]
    rng = np.random.default_rng(3)
    cuts = sorted([0, len(ps)] + [int(c) for c in rng.integers(0, len(ps), 4)] + [len(ps) // 2] * 2)  # one empty piece
    s = 0.0
    for a, b in zip(cuts[:-1], cuts[1:]):
        s, _ = engine(ps[a:b], s0=s)
    assert bits(s) == bits(seqsum(ps))


def test_engine_takes_the_fast_path():
    """Where the guesses are good the sub-segment maps apply (the walk is not the serial sum in disguise)."""
    for name in ("walk", "ties_even", "ties_odd", "quarter", "drift", "small_on_large"):
        ps = [float(v) for v in CASES[name]]
        _, fast = engine(ps)
        assert fast > len(ps) // 16 // 4, (name, fast)


@pytest.mark.parametrize("name", ["ties_even", "ties_odd", "walk", "drift"])
def test_composition_is_associative(name):
    """Left fold, right fold and a balanced tree of 16 lane runs are the same map (the kernel composes in trees
    and wave scans); it applies to the actual start exactly when the whole run stays in the binade."""
    ps = [float(v) for v in CASES[name][:256]]
    s0 = seqsum(ps[:1])
    gok, e, sn = guess(s0)
    lanes = [run(ps[1 + 15 * k:1 + 15 * (k + 1)], e, sn, gok) for k in range(16)]
    left = lanes[0]
    for u in lanes[1:]:
        left = comb(left, u)
    right = lanes[-1]
    for u in reversed(lanes[:-1]):
        right = comb(u, right)
    tree = lanes
    while len(tree) > 1:
        tree = [comb(tree[i], tree[i + 1]) for i in range(0, len(tree), 2)]
    for t in (right, tree[0]):
        assert {k: t[k] for k in ("d", "lo", "hi", "bad")} == {k: left[k] for k in ("d", "lo", "hi", "bad")}
    r = apply(left, s0)
    if r is not None:
        assert bits(r) == bits(seqsum(ps[1:241], s0))


def decomp_f(p, e, sneg):
    """k_seqx_trans's f64 decomposition: a = |p| * 2^(52-e) by ldexp, its exact floor and fraction."""
    if not math.isfinite(p):
        return None
    try:
        a = math.ldexp(abs(p), 52 - e)
    except OverflowError:  # the device's ldexp gives inf, which the next test refuses
        return None
    if a >= 2.0 ** 53:
        return None
    qa = math.floor(a)
    fa = a - qa
    neg = (1 if math.copysign(1.0, p) < 0 else 0) != sneg
    if not neg:
        return qa, (2 if fa > 0.5 else (1 if fa == 0.5 else 0))
    if fa == 0.0:
        return -qa, 0
    return -qa - 1, (2 if fa < 0.5 else (1 if fa == 0.5 else 0))


def test_f64_decomposition_equals_the_integer_one():
    """The device decomposes terms in f64; it must give decomp's (q, class) for every term the walk can meet,
    including halves and near-halves of the state's ulp, subnormals, terms far below the ulp and terms at 2^(e+1)."""
    rng = np.random.default_rng(7)
    es = [-1022, -1000, -300, -60, -5, 0, 1, 30, 52, 53, 200, 1023]
    for e in es:
        u = 2.0 ** (e - 52) if e - 52 >= -1074 else 0.0
        ps = list(rng.standard_normal(300) * 2.0 ** e)
        ps += list(rng.standard_normal(300) * 2.0 ** (e - 40))
        if u:
            for k in range(1, 60):
                for m in (1, 3, 5):
                    h = u * m / 2.0 ** k
                    ps += [h, -h, math.nextafter(h, 0.0), -math.nextafter(h, 0.0), math.nextafter(h, math.inf)]
        ps += [2.0 ** e, -(2.0 ** e), 2.0 ** (e + 1) if e < 1023 else math.inf, 5e-324, -5e-324, 2.2e-308,
               math.nextafter(2.0 ** (e + 1), 0.0) if e < 1023 else 1.0, math.inf, -math.inf, math.nan]
        for p in ps:
            for sneg in (0, 1):
                if p == 0.0:
                    continue
                r_int, r_f = decomp(p, e, sneg), decomp_f(p, e, sneg)
                if r_int is None or r_f is None:
                    assert r_int is None and r_f is None, (p, e, sneg, r_int, r_f)
                elif r_int != (int(r_f[0]), r_f[1]):
                    # the one benign difference: a negative term so far below the ulp that |p| * 2^(52-e)
                    # underflows to 0.  decomp says (floor -1, fraction > 1/2), decomp_f says (0, 0): the same
                    # increment (0, the state is unchanged, as the f64 add rounds it), and a lowest exact sum one
                    # unit higher, which is exact in the only case it decides (s = 2^e: RN(2^e - tiny) = 2^e).
                    assert r_int == (-1, 2) and r_f == (0, 0) and math.ldexp(abs(p), 52 - e) == 0.0, \
                        (p, e, sneg, r_int, r_f)


def _ldexp(x, sh):
    try:
        return math.ldexp(float(x), sh)
    except OverflowError:
        return math.inf if x > 0 else -math.inf


def prep(t):
    """k_seqx_walk's prepared map (Prep, round 5): in the map's binade the valid states are |s| in [L_p, H_p) of the
    map's sign, and the result is |s| + d_p u, one f64 add."""
    if t["zero"]:
        return dict(zero=True, nzero=t["nzero"])
    sh = t["e"] - 52
    L = [_ldexp(max(M0, M0 - t["lo"][p]), sh) for p in (0, 1)]
    H = [_ldexp(min(M1, M1 - t["hi"][p]), sh) for p in (0, 1)]
    D = [_ldexp(t["d"][p], sh) for p in (0, 1)]
    if t["bad"]:
        L = [math.inf, math.inf]
    return dict(zero=False, L=L, H=H, D=D, neg=t["neg"])


def prep_apply(q, s):
    if q["zero"]:
        if s == 0.0:
            return -0.0 if (math.copysign(1.0, s) < 0 and q["nzero"]) else 0.0
        return s
    b = bits(s)
    od, neg, a = b & 1, b >> 63, abs(s)
    if not (a >= q["L"][od] and a < q["H"][od] and neg == q["neg"]):
        return None
    m = a + q["D"][od]
    return -m if neg else m


@pytest.mark.parametrize("name", list(CASES))
def test_prepared_map_apply_is_tr_apply(name):
    """The walk's one-record applies on prepared maps decide and compute exactly as tr_apply: for every sub-segment
    map of the case (built in the binade of the true and of a jittered guess) and every state the sequential sum
    passes through near it (and +-0, subnormals, +-inf), the same verdict and the same bits."""
    ps = [float(v) for v in CASES[name]]
    pre = [0.0]
    for p in ps:
        pre.append(pre[-1] + p)
    rng = np.random.default_rng(11)
    extra = [0.0, -0.0, 5e-324, -5e-324, math.inf, -math.inf, 1.0, -1.0]
    checked = 0
    for i in range(0, len(ps), 16):
        for G in (pre[i], pre[i] * (1.0 + 1e-9 * rng.uniform(-1, 1))):
            gok, e, sn = guess(G)
            t = run(ps[i:i + 16], e, sn, gok)
            q = prep(t)
            for s in [pre[i], pre[min(i + 1, len(ps))], pre[min(i + 16, len(ps))]] + extra:
                r1, r2 = apply(t, s), prep_apply(q, s)
                assert (r1 is None) == (r2 is None), (name, i, s, r1, r2)
                if r1 is not None:
                    assert bits(r1) == bits(r2), (name, i, s, r1, r2)
                    checked += 1
    assert checked > 0 or name in ("inf", "overflow", "neg_zero", "cancel", "subnormal")

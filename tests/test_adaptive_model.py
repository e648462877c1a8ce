"""CPU checks of the two facts the adaptive random kernels (fl_sim_amd/csrc/adaptive.hip) rest on.

1. numpy's order for ``np.abs(x).sum()`` on a contiguous fp32 vector: the reduction runs over buffers of
   np.getbufsize() = 8192 elements folded in order, each buffer summed by ``pairwise_sum`` (leaves of at
   most 128 elements with 8 accumulators; splits at n/2 rounded down to a multiple of 8).  Restated here
   and compared with numpy itself, bit for bit.
2. The speculated fp64 running sum: a chunk's sequential run from a guess g shifted by (t - g) equals the
   run from the true start t whenever (t - g) is an even multiple of the binade's spacing and both stay in
   one binade (round-to-nearest-even commutes with such shifts).  The kernel's phase A / phase B scheme
   is modelled here with numpy (vectorised across chunks) and must reproduce ``np.cumsum`` exactly at every
   chunk boundary, re-running only a few chunks.
"""

import math
import sys

import numpy as np
import pytest

sys.setrecursionlimit(10_000)
F32 = np.float32


def pairwise_sum(a: np.ndarray) -> np.float32:
    n = len(a)
    if n < 8:
        r = F32(0)
        for v in a:
            r = F32(r + v)
        return r
    if n <= 128:
        r = [F32(v) for v in a[:8]]
        i = 8
        while i < n - (n % 8):
            for j in range(8):
                r[j] = F32(r[j] + a[i + j])
            i += 8
        res = F32(F32(F32(r[0] + r[1]) + F32(r[2] + r[3])) + F32(F32(r[4] + r[5]) + F32(r[6] + r[7])))
        for v in a[i:]:
            res = F32(res + v)
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return F32(pairwise_sum(a[:n2]) + pairwise_sum(a[n2:]))


def numpy_order_sum(a: np.ndarray) -> np.float32:
    s = F32(0)
    for b in range(0, len(a), 8192):
        s = F32(s + pairwise_sum(a[b:b + 8192]))
    return s


@pytest.mark.parametrize("n", [1, 5, 8, 9, 127, 128, 129, 300, 1000, 8191, 8192, 8193, 16384, 20_000, 65_537])
@pytest.mark.parametrize("scale", [1e-3, 1.0, 3e5])
def test_numpy_sum_order(n, scale):
    g = np.random.default_rng(n)
    x = np.abs((g.standard_normal(n) * scale).astype(F32))
    assert np.getbufsize() == 8192
    assert numpy_order_sum(x).view(np.uint32) == np.abs(x).sum().view(np.uint32)


def _binade(v: float) -> int:
    return int(np.float64(v).view(np.uint64) >> np.uint64(52))


def _spacing(e: int) -> float:
    return 5e-324 if e == 0 else math.ldexp(1.0, e - 1075)


def speculated_cumsum_ends(p: np.ndarray, chunk: int, guess: np.ndarray):
    """The kernel's scheme: returns (exact running sum at each chunk end, number of re-run chunks)."""
    n = len(p)
    nq = -(-n // chunk)
    P = np.zeros(nq * chunk)
    P[:n] = p
    P = P.reshape(nq, chunk)
    ga = guess.astype(np.float64)
    gb = np.array([g + _spacing(_binade(g)) for g in ga])
    ea, eb = ga.copy(), gb.copy()
    for s in range(chunk):  # phase A: every chunk's two runs, in parallel across chunks
        ea = ea + P[:, s]
        eb = eb + P[:, s]
    t, reruns, ends = 0.0, 0, []
    for j in range(nq):  # phase B
        d = t - ga[j]
        if d == 0.0:
            t = ea[j]
        else:
            e = _binade(ga[j])
            ok = e > 64 and _binade(t) == e
            if ok:
                k = d * math.ldexp(1.0, 1075 - e)
                even = int(k) % 2 == 0
                g, end = (ga[j], ea[j]) if even else (gb[j], eb[j])
                cand = end + (t - g)
                ok = _binade(g) == e and _binade(end) == e and _binade(cand) == e
            if ok:
                t = cand
            else:
                reruns += 1
                for q in P[j]:
                    t = t + q
        ends.append(t)
    return np.array(ends), reruns


@pytest.mark.parametrize("n,dist,zero_frac", [(1 << 18, "normal", 0.0), (1_000_003, "normal", 0.05),
                                              (1 << 20, "cauchy", 0.2), (300_001, "lognormal", 0.5),
                                              (200_000, "spiky", 0.0)])
def test_speculated_cumsum_is_exact(n, dist, zero_frac):
    g = np.random.default_rng(n)
    if dist == "normal":
        x = g.standard_normal(n)
    elif dist == "cauchy":
        x = g.standard_cauchy(n)
    elif dist == "lognormal":
        x = g.lognormal(0, 8, n)  # many binades apart
    else:
        x = g.standard_normal(n) * 1e-6
        x[g.integers(0, n, 20)] = 1e3  # a handful of elements carry nearly all the mass
    x = x.astype(F32)
    x[g.random(n) < zero_frac] = 0
    ax = np.abs(x)
    p = (ax / ax.sum()).astype(np.float64)
    chunk = 2048
    starts = np.arange(0, n, chunk)
    q = np.add.reduceat(ax.astype(np.float64), starts)
    guess = np.concatenate([[0.0], np.cumsum(q)[:-1]]) / float(ax.sum())
    ends, reruns = speculated_cumsum_ends(p, chunk, guess)
    cdf = np.cumsum(p)
    want = cdf[np.minimum(starts + chunk, n) - 1]
    assert np.array_equal(ends, want)
    assert reruns <= 80  # about one per binade the running sum crosses


def _compose(f, g):
    """f then g on (increment for an even start, increment for an odd start)."""
    h0 = f[0] + (g[1] if f[0] & 1 else g[0])
    h1 = f[1] + (g[0] if f[1] & 1 else g[1])
    return h0, h1


def _apply(m, f):
    return m + (f[1] if m & 1 else f[0])


def special_map(row: np.ndarray, ga: float, e: int):
    """adaptive.hip K3b: a chunk whose speculated runs cross into binade e + 1 or come near an edge, run from the
    guess's grid index G + r (r = 0..3).  Per run: its end (grid index of binade e + cross), whether it crossed, and the
    largest |d| (in spacings of binade e) for which the run shifted by d (d = 0 mod 4) is the run from G + r + d."""
    G = int(math.ldexp(ga, 1075 - e))
    edge = math.ldexp(1.0, e - 1022)
    out = []
    for r in range(4):
        t0 = math.ldexp(float(G + r), e - 1075)
        if not (1 << 52) <= G + r < (1 << 53):
            out.append((0, 0, -1))
            continue
        t, below, above = t0, t0, math.inf
        for q in row:
            t = t + q
            if t < edge:
                below = t
            elif t < above:
                above = t
        eb = _binade(t)
        if eb == e:
            out.append((int(math.ldexp(t, 1075 - e)), 0, int(math.ldexp(edge - t, 1075 - e)) - 2))
        elif eb == e + 1:
            lo = int(math.ldexp(edge - below, 1075 - e))
            hi = int(math.ldexp(above - edge, 1075 - e))
            top = int(math.ldexp(2.0 * edge - t, 1075 - e))
            out.append((int(math.ldexp(t, 1074 - e)), 1, min(lo, hi, top) - 2))
        else:
            out.append((0, 0, -1))
    return G, out


def special_apply(t: float, e: int, G: int, runs):
    """The walk's step over a special chunk: the exact end, or None (re-run the chunk)."""
    if _binade(t) != e:
        return None
    m = int(math.ldexp(t, 1075 - e))
    r = (m - G) & 3
    d = m - G - r
    end, cross, margin = runs[r]
    if margin < 0 or abs(d) > margin:
        return None
    return math.ldexp(float(end + d // 2), e + 1 - 1075) if cross else math.ldexp(float(end + d), e - 1075)


def parallel_cumsum_starts(p: np.ndarray, chunk: int, guess: np.ndarray, piece_blk: int = 1024,
                           rec_max: int = 128, eta: float = 2.0 ** -16, specials: bool = True):
    """The kernels' current scheme (adaptive.hip K3, K3b, K5-K7): per-chunk parity maps from the two speculated runs,
    composed inside pieces of one binade per scan block; the chunks whose runs cross into the next binade or come near
    an edge get a four-run map of their own (K3b); a walk over the pieces (re-running the chunks whose maps are
    unusable for the true start) and every chunk's start from its piece's start and its exclusive prefix map.  Returns
    (exact start of every chunk + the total, number of re-run chunks) or None where the kernels take the sequential
    chain.  specials=False: the round-3 scheme before K3b (every such chunk re-run)."""
    n = len(p)
    nq = -(-n // chunk)
    P = np.zeros(nq * chunk)
    P[:n] = p
    P = P.reshape(nq, chunk)
    ga = guess.astype(np.float64)
    E = np.array([_binade(g) for g in ga])
    gb = np.array([g + _spacing(int(e)) for g, e in zip(ga, E)])
    ea, eb = ga.copy(), gb.copy()
    for s in range(chunk):
        ea = ea + P[:, s]
        eb = eb + P[:, s]
    fe, fn, spec = [], [], []
    for j in range(nq):
        e = int(E[j])
        ok = (e >= 1 and _binade(gb[j]) == e and _binade(ea[j]) == e and _binade(eb[j]) == e
              and ga[j] >= math.ldexp(1.0 + eta, e - 1023) and max(ea[j], eb[j]) <= math.ldexp(1.0 - eta, e - 1022))
        if ok:
            G = int(math.ldexp(ga[j], 1075 - e))
            d0, d1 = int(math.ldexp(ea[j] - ga[j], 1075 - e)), int(math.ldexp(eb[j] - gb[j], 1075 - e))
            fn.append((d1, d0) if G & 1 else (d0, d1))
        else:
            fn.append((0, 0))
        if ok:
            fe.append(e)
        elif specials and 1 <= e <= 2045 and _binade(ea[j]) <= e + 1:
            fe.append(-2 - len(spec))
            spec.append(special_map(P[j], float(ga[j]), e))
        else:
            fe.append(-1)
    # pieces (K5) and their prefix maps
    pieces, pre, piece_of = [], [None] * nq, [0] * nq
    for b0 in range(0, nq, piece_blk):
        nb = 0
        for j in range(b0, min(nq, b0 + piece_blk)):
            head = j == b0 or fe[j] < 0 or fe[j - 1] < 0 or fe[j] != fe[j - 1]
            if head:
                pieces.append([j, fe[j], (0, 0)])
                nb += 1
            pre[j] = pieces[-1][2]
            pieces[-1][2] = _compose(pieces[-1][2], fn[j])
            piece_of[j] = len(pieces) - 1
        if nb > rec_max:
            return None
    # the walk (K6)
    t, reruns, tstart = 0.0, 0, []
    for first, e, f in pieces:
        tstart.append(t)
        if e >= 1:
            if _binade(t) != e:
                return None
            m = _apply(int(math.ldexp(t, 1075 - e)), f)
            if not (1 << 52) <= m < (1 << 53):
                return None
            t = math.ldexp(float(m), e - 1075)
        elif t == ga[first]:
            t = ea[first]
        elif e <= -2 and (nt := special_apply(t, int(E[first]), *spec[-2 - e])) is not None:
            t = nt
        else:
            reruns += 1
            for q in P[first]:
                t = t + q
    # the fill (K7)
    starts = []
    for j in range(nq):
        tp = tstart[piece_of[j]]
        starts.append(math.ldexp(float(_apply(int(math.ldexp(tp, 1075 - fe[j])), pre[j])), fe[j] - 1075)
                      if fe[j] >= 1 else tp)
    return np.array(starts + [t]), reruns


@pytest.mark.parametrize("n,dist,zero_frac", [(1 << 18, "normal", 0.0), (1_000_003, "normal", 0.05),
                                              (1 << 20, "cauchy", 0.2), (300_001, "lognormal", 0.5),
                                              (200_000, "spiky", 0.0), (300_000, "sparse", 0.0)])
def test_parallel_cumsum_is_exact(n, dist, zero_frac):
    g = np.random.default_rng(n + 1)
    if dist == "normal":
        x = g.standard_normal(n)
    elif dist == "cauchy":
        x = g.standard_cauchy(n)
    elif dist == "lognormal":
        x = g.lognormal(0, 8, n)
    elif dist == "spiky":
        x = g.standard_normal(n) * 1e-6
        x[g.integers(0, n, 20)] = 1e3
    else:
        x = np.zeros(n)
        x[g.integers(0, n, 50)] = g.standard_normal(50)
    x = x.astype(F32)
    x[g.random(n) < zero_frac] = 0
    ax = np.abs(x)
    S = ax.sum()
    p = (ax / S).astype(np.float64)
    chunk = 256
    starts = np.arange(0, n, chunk)
    q = np.add.reduceat(ax.astype(np.float64), starts)
    guess = np.concatenate([[0.0], np.cumsum(q)[:-1]]) / float(S)
    res = parallel_cumsum_starts(p, chunk, guess)
    assert res is not None  # the speculation verifies on all of these
    got, reruns = res
    cdf = np.cumsum(p)
    want = np.concatenate([[0.0], cdf[starts[1:] - 1], [cdf[-1]]])
    assert np.array_equal(got, want)
    assert reruns <= 3  # the special chunks' maps serve nearly every binade crossing
    _, reruns_before = parallel_cumsum_starts(p, chunk, guess, specials=False)
    assert reruns_before <= 80


@pytest.mark.parametrize("noise", [1e-13, 1e-10, 1e-7])
def test_special_maps_stay_exact_under_poor_guesses(noise):
    """Guesses perturbed far beyond the kernels' own error: every special map that is taken must still give the exact
    run (the margins fail over to a re-run, never to a wrong sum)."""
    n = 400_000
    g = np.random.default_rng(7)
    x = g.standard_normal(n).astype(F32)
    ax = np.abs(x)
    S = ax.sum()
    p = (ax / S).astype(np.float64)
    starts = np.arange(0, n, 256)
    q = np.add.reduceat(ax.astype(np.float64), starts)
    guess = np.concatenate([[0.0], np.cumsum(q)[:-1]]) / float(S)
    guess[1:] *= 1.0 + noise * g.standard_normal(len(guess) - 1)
    res = parallel_cumsum_starts(p, 256, guess, eta=2.0 ** -30)
    assert res is not None
    got, _ = res
    cdf = np.cumsum(p)
    want = np.concatenate([[0.0], cdf[starts[1:] - 1], [cdf[-1]]])
    assert np.array_equal(got, want)


def test_special_map_crossing_shifts_exhaustive():
    """One crossing chunk, every true start within +-64 spacings of the guess: the map, where it answers, equals the
    sequential run from that start."""
    g = np.random.default_rng(3)
    row = np.abs(g.standard_normal(256)) * 2.0 ** -20
    e = _binade(0.5)
    edge = 1.0
    ga = edge - 100.5 * 2.0 ** -20  # the run crosses 1.0 about half-way
    ga = math.ldexp(float(int(math.ldexp(ga, 1075 - e))), e - 1075)
    G, runs = special_map(row, ga, e)
    assert all(c == 1 for _, c, _ in runs)
    answered = 0
    for dm in range(-64, 65):
        t0 = math.ldexp(float(G + dm), e - 1075)
        want = t0
        for v in row:
            want = want + v
        got = special_apply(t0, e, G, runs)
        if got is not None:
            answered += 1
            assert got == want, dm
    assert answered == 129


def test_parallel_cumsum_many_binades_takes_the_sequential_chain():
    """Exponentially growing magnitudes cross a binade in nearly every chunk: more pieces than a scan block keeps,
    so the kernels run the exact sequential chain instead (the model returns None there)."""
    n = 100_000
    x = np.exp2(np.arange(n) / 1000.0).astype(F32)  # doubles every ~4 chunks
    ax = np.abs(x)
    p = (ax / ax.sum()).astype(np.float64)
    starts = np.arange(0, n, 256)
    q = np.add.reduceat(ax.astype(np.float64), starts)
    guess = np.concatenate([[0.0], np.cumsum(q)[:-1]]) / float(ax.sum())
    res = parallel_cumsum_starts(p, 256, guess, piece_blk=64, rec_max=8)
    assert res is None

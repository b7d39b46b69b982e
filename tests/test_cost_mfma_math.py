"""Host-side check of the arithmetic k_cost_mfma relies on (csrc/k_cost.hip).

1. The ternary census of ADCensus.cpp:454-498 as the device walk computes it,
   sum_w popc((F[w] & V[6+w]) | (F[6+w] & V[w])) over the 6 gt / 6 lt words, equals the
   dot product of the 384 record bits with the varying record's halves swapped,
   sum_w popc(F[w] & V[(w+6) % 12]) -- because a neighbour is never both gt and lt.
2. The fp4 expansion (bit 4n+s of a word -> nibble n of dword s, 0x4 = e2m1 2.0) puts
   every bit at one slot of the 16-B fragment, so the slot-wise product sum of two
   expanded words is 4 x popc(a & b): the byte offset of the census table entry.
"""
import numpy as np


def _ternary_records(rng, n):
    # 3 channels x 62 neighbours: -1 / 0 / +1 per (channel, neighbour)
    t = rng.integers(-1, 2, size=(n, 3, 62))
    words = np.zeros((n, 12), np.uint64)
    for c in range(3):
        for b in range(62):
            w, bit = divmod(b, 32)
            words[:, 2 * c + w] |= (t[:, c, b] > 0).astype(np.uint64) << np.uint64(bit)
            words[:, 6 + 2 * c + w] |= (t[:, c, b] < 0).astype(np.uint64) << np.uint64(bit)
    return t, words.astype(np.uint32)


def _popc(x):
    x = np.asarray(x, np.uint64)
    return np.array([bin(int(v)).count("1") for v in x.ravel()]).reshape(x.shape)


def test_census_is_a_dot_product_of_swapped_halves():
    rng = np.random.default_rng(5)
    tf, F = _ternary_records(rng, 200)
    tv, V = _ternary_records(rng, 200)
    walk = sum(_popc((F[:, w] & V[:, 6 + w]) | (F[:, 6 + w] & V[:, w])) for w in range(6))
    dot = sum(_popc(F[:, w] & V[:, (w + 6) % 12]) for w in range(12))
    ref = ((tf * tv) < 0).sum(axis=(1, 2))  # the reference's sign-product count
    assert np.array_equal(walk, ref)
    assert np.array_equal(dot, ref)


def _fp4_expand(w):
    w = np.uint32(w)
    m = np.uint32(0x44444444)
    d = [(w << np.uint32(2)) & m, (w << np.uint32(1)) & m, w & m, (w >> np.uint32(1)) & m]
    # 32 nibbles (slot = 8 * dword + nibble), e2m1 value: 0x4 -> 2.0, 0 -> 0.0
    nib = np.array([(int(d[s]) >> (4 * n)) & 0xF for s in range(4) for n in range(8)])
    assert set(np.unique(nib)) <= {0, 4}
    return np.where(nib == 4, 2.0, 0.0)


def test_fp4_fragment_dot_is_four_popcounts():
    rng = np.random.default_rng(9)
    for _ in range(300):
        a, b = (int(x) for x in rng.integers(0, 1 << 32, size=2, dtype=np.uint64))
        ea, eb = _fp4_expand(a), _fp4_expand(b)
        assert ea.sum() == 2.0 * bin(a).count("1")  # every bit lands in exactly one slot
        assert float(ea @ eb) == 4.0 * bin(a & b).count("1")
    full = _fp4_expand(0xFFFFFFFF)
    assert float(full @ full) * 12 == 4.0 * 384  # 12 words: the f32 sum stays exact (1536)

"""CPU: the entropy-coder restatements. compressai is absent, so the coder
is pinned by hand-worked known answers, Python == C byte equality, product-table == oracle-table
equality and round trips (parity vs compressai itself is unpinned).

The product's quantiser (fvc_pmf_to_quantized_cdf, host C++ in libfvc) edits the cumulative
table in place as ops.cpp does; the oracle's numpy and C quantisers work on the frequency array
(oracle/rans_ref.c header), so table equality here compares two different programs."""
import numpy as np
import pytest

from fastvideocodec_amd import entropy_models as EM
from oracle import coder_ref as R


def test_pmf_known_answers():
    # uniform over 4: 16384 each
    assert R.pmf_to_quantized_cdf_py([0.25] * 4).tolist() == [0, 16384, 32768, 49152, 65536]
    # a zero-probability bin steals one count from the lowest bin with freq > 1
    assert R.pmf_to_quantized_cdf_py([0.5, 0.0, 0.5]).tolist() == [0, 32767, 32768, 65536]
    # rounding is half away from zero on the float32 product, then renormalised by the total
    assert R.pmf_to_quantized_cdf_py([1.0, 1.0]).tolist() == [0, 32768, 65536]
    with pytest.raises(ValueError):
        R.pmf_to_quantized_cdf_py([0.5, -0.1])
    with pytest.raises(ValueError):
        R.pmf_to_quantized_cdf_py([0.0, 0.0])


def test_rans_known_answer():
    """Two symbols, table {0: [0,32767), 1: [32767,65534), escape: [65534,65536)}: hand-run of
    Rans64EncPut (x0 = 2^31, symbols put in reverse order) and Rans64EncFlush ([lo, hi] words)."""
    cdf = np.array([[0, 32767, 65534, 65536]], np.int32)
    sizes = np.array([4], np.int32)
    offsets = np.array([0], np.int32)
    s = R.rans_encode_py([0, 1], [0, 0], cdf, sizes, offsets)
    words = np.frombuffer(s, "<u4")
    # recompute by hand with the same formulas (independent of the helper)
    x = 1 << 31
    for start, freq in [(32767, 32767), (0, 32767)]:   # reverse order: symbol 1 first, then 0
        x = ((x // freq) << 16) + (x % freq) + start
    assert words.tolist() == [x & 0xFFFFFFFF, x >> 32]
    assert R.rans_decode_py(s, [0, 0], cdf, sizes, offsets) == [0, 1]


@pytest.fixture(scope="module")
def lap():
    return EM.LaplaceTables()


@pytest.mark.parametrize("quantizer", ["numpy", "c"])
def test_tables_product_equals_oracle(seeded_sd, lap, quantizer):
    """Every real table (64 Laplace scales, 64 z channels, 128 mv channels) built by the product
    equals the oracle's, with the oracle quantising by its numpy or its C restatement."""
    q = R.pmf_to_quantized_cdf_np if quantizer == "numpy" else R.CRef.pmf_to_quantized_cdf
    c, l, o = R.laplace_tables(lap.scale_table, quantize=q)
    assert (c == lap.cdf).all() and (l == lap.cdf_length).all() and (o == lap.offset).all()
    assert c.shape[0] == 64
    for name, ch in (("bitEstimator_z", 64), ("bitEstimator_mv", 128)):
        rows = [seeded_sd[f"{name}.f{f}.{p}"].numpy().reshape(-1) for f in (1, 2, 3) for p in "hba"]
        rows += [seeded_sd[f"{name}.f4.h"].numpy().reshape(-1), seeded_sd[f"{name}.f4.b"].numpy().reshape(-1)]
        prm = np.stack(rows)
        ft = EM.FactorizedTables(prm)
        c, l, o = R.factorized_tables(prm, quantize=q)
        assert (c == ft.cdf).all() and (l == ft.cdf_length).all() and (o == ft.offset).all()
        assert ft.cdf.shape[0] == ch


def test_quantizers_agree_on_random_pmfs():
    """Loop restatement (ops.cpp literally) == numpy (frequency array) == C oracle == product, on
    pmfs with empty bins, ties and heavy tails (the repair path)."""
    rng = np.random.default_rng(1)
    for _ in range(300):
        n = int(rng.integers(1, 60))
        p = rng.random(n) ** int(rng.integers(1, 30))
        p[rng.random(n) < 0.3] = 0
        if p.sum() == 0:
            p[0] = 1
        p = (p / p.sum()).astype(np.float32)
        a = R.pmf_to_quantized_cdf_py(p)
        b = R.pmf_to_quantized_cdf_np(p)
        c = R.CRef.pmf_to_quantized_cdf(p)
        d = EM.pmf_to_quantized_cdf(p)
        assert a.tolist() == b.tolist() == c.tolist() == d.tolist(), p


def test_tables_are_valid_cdfs(lap):
    for i in range(lap.cdf.shape[0]):
        n = lap.cdf_length[i]
        row = lap.cdf[i, :n]
        assert row[0] == 0 and row[-1] == 65536 and (np.diff(row) > 0).all()


def test_scale_table_and_indexes():
    st = EM.get_scale_table().numpy()
    assert st.shape == (64,) and abs(st[0] - 0.11) < 1e-6 and abs(st[-1] - 256) < 1e-3
    idx = R.build_indexes(np.array([0.01, 0.11, 0.1101, 255.0, 1e9], np.float32), st)
    assert idx.tolist()[0] == 0 and idx.tolist()[1] == 0 and idx.tolist()[-1] == 63


@pytest.mark.parametrize("seed", range(4))
def test_py_equals_c_and_roundtrip(lap, seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 400))
    sym = np.round(rng.laplace(0, 5, n)).astype(np.int32)
    sym[rng.integers(0, n, max(1, n // 40))] = rng.integers(-2 ** 20, 2 ** 20, max(1, n // 40))
    idx = rng.integers(0, 64, n).astype(np.int32)
    a = R.rans_encode_py(sym, idx, lap.cdf, lap.cdf_length, lap.offset)
    b = R.CRef.encode(sym, idx, lap.cdf, lap.cdf_length, lap.offset)
    assert a == b
    assert (R.CRef.decode(b, idx, lap.cdf, lap.cdf_length, lap.offset) == sym).all()
    assert R.rans_decode_py(a, idx, lap.cdf, lap.cdf_length, lap.offset) == sym.tolist()


def test_empty_stream(lap):
    s = R.rans_encode_py([], [], lap.cdf, lap.cdf_length, lap.offset)
    assert len(s) == 8  # just the flushed state
    assert R.rans_decode_py(s, [], lap.cdf, lap.cdf_length, lap.offset) == []


def test_extreme_escapes(lap):
    sym = np.array([0, 2 ** 30, -2 ** 30, 12345678, -1, 7], np.int32)
    idx = np.array([0, 63, 0, 31, 5, 9], np.int32)
    b = R.CRef.encode(sym, idx, lap.cdf, lap.cdf_length, lap.offset)
    assert (R.CRef.decode(b, idx, lap.cdf, lap.cdf_length, lap.offset) == sym).all()


def test_gaussian_tables_product_equals_oracle():
    """compressai GaussianConditional tables (RLVC's RPM path) over get_scale_table()."""
    g = EM.GaussianTables()
    c, l, o = R.gaussian_tables(EM.get_scale_table().numpy())
    assert (c == g.cdf).all() and (l == g.cdf_length).all() and (o == g.offset).all()
    assert g.cdf_length[0] == 5 and g.offset[0] == -1  # scale 0.11: centre ceil(0.11 * 6.109) = 1

"""CPU: the bitstream coder (csrc/rans.cpp via rgbac.ans) and the CDF tables against the
oracle restatement of compressai's algorithm (oracle/ans_ref.py), plus hand-derived known
answers.  Parity at the compressai boundary is unpinned (compressai absent, no reference
fixtures): the known answers below are derived by hand from the published rans64 / ops.cpp
arithmetic, and everything else is byte-exact agreement with the oracle and round trips."""
import numpy as np
import pytest
import torch

from oracle import ans_ref as oa


def _tables(rng, n_tables=6, max_len=40):
    cdfs, lens, offs = [], [], []
    for _ in range(n_tables):
        L = int(rng.integers(2, max_len))
        pmf = rng.random(L).astype(np.float32) ** 3
        pmf = pmf / pmf.sum() * np.float32(0.999)
        prob = list(pmf) + [np.float32(0.001)]
        c = oa.pmf_to_quantized_cdf(prob)
        cdfs.append(c)
        lens.append(len(c))
        offs.append(-int(rng.integers(0, L)))
    width = max(lens)
    tab = [c + [0] * (width - len(c)) for c in cdfs]
    return tab, lens, offs


def test_pmf_to_quantized_cdf_known_answers():
    from rgbac.ans import pmf_to_quantized_cdf
    # exact quantisation: [1/2, 1/4, 1/4] -> 0, 32768, 49152, 65536
    assert pmf_to_quantized_cdf([0.5, 0.25, 0.25]) == [0, 32768, 49152, 65536]
    # a zero-probability symbol gets one count stolen from the first smallest frequency > 1
    # (symbol 2, 16384 -> 16383, which lies after it: cdf[2] += 1)
    assert pmf_to_quantized_cdf([0.5, 0.0, 0.25, 0.25]) == [0, 32768, 32769, 49152, 65536]
    # ... and from before it when the donor precedes: cdf[1..2] -= 1
    assert pmf_to_quantized_cdf([0.25, 0.75, 0.0]) == [0, 16383, 65535, 65536]
    for pmf in ([0.5, 0.0, 0.25, 0.25], [1e-7, 0.3, 0.7, 0.0, 0.0], [0.2] * 5):
        assert pmf_to_quantized_cdf(pmf) == oa.pmf_to_quantized_cdf(pmf)


def test_pmf_to_quantized_cdf_random_matches_oracle():
    from rgbac.ans import pmf_to_quantized_cdf
    rng = np.random.default_rng(0)
    for _ in range(50):
        L = int(rng.integers(1, 300))
        pmf = (rng.random(L) ** 6).astype(np.float32)
        pmf[rng.random(L) < 0.2] = 0.0
        if pmf.sum() == 0:
            pmf[0] = 1.0
        pmf = pmf / pmf.sum()
        assert pmf_to_quantized_cdf(pmf) == oa.pmf_to_quantized_cdf(pmf.tolist())


def test_pmf_to_quantized_cdf_rejects_bad_pmf():
    from rgbac.ans import pmf_to_quantized_cdf
    with pytest.raises(RuntimeError, match="non-finite or negative"):
        pmf_to_quantized_cdf([0.5, -0.1, 0.6])
    with pytest.raises(RuntimeError, match="non-zero"):
        pmf_to_quantized_cdf([0.0, 0.0])


def test_one_symbol_stream_known_answer():
    # cdf [0, 32768, 65536] (two equiprobable symbols, escape is symbol 1 -> size 3):
    # state L = 2^31; encode s=0: x = ((2^31 // 32768) << 16) + 0 + 0 = 2^32 -> flush writes
    # lo = 0, hi = 1: bytes 00000000 01000000.  s=0 with start 0 / freq 32768.
    from rgbac.ans import RansDecoder, RansEncoder
    cdfs, lens, offs = [[0, 32768, 65536]], [3], [0]
    s = RansEncoder().encode_with_indexes([0], [0], cdfs, lens, offs)
    assert s == bytes([0, 0, 0, 0, 1, 0, 0, 0])
    assert oa.BufferedRansEncoder().flush() == bytes([0, 0, 0, 128, 0, 0, 0, 0])  # empty: L
    assert RansDecoder().decode_with_indexes(s, [0], cdfs, lens, offs) == [0]


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_rans_matches_oracle_bytes_and_round_trips(seed):
    from rgbac.ans import BufferedRansEncoder, RansDecoder
    rng = np.random.default_rng(seed)
    tab, lens, offs = _tables(rng)
    n = 3000
    idx = rng.integers(0, len(tab), n).astype(np.int32)
    # mostly in-range symbols, some far outside (bypass coding, both signs, long digit runs)
    sym = np.array([int(rng.integers(offs[i], offs[i] + lens[i] - 2)) for i in idx], np.int32)
    far = rng.random(n) < 0.05
    sym[far] = rng.integers(-(1 << 20), 1 << 20, far.sum())
    sym[:3] = [offs[idx[0]] + lens[idx[0]] - 2, offs[idx[1]] - 1, (1 << 30)]  # edges
    enc = BufferedRansEncoder()
    enc.encode_with_indexes(sym[:1000].tolist(), idx[:1000].tolist(), tab, lens, offs)
    enc.encode_with_indexes(sym[1000:], idx[1000:], tab, lens, offs)   # numpy accepted
    got = enc.flush()
    o = oa.BufferedRansEncoder()
    o.encode_with_indexes(sym.tolist(), idx.tolist(), tab, lens, offs)
    assert got == o.flush()
    d = RansDecoder()
    d.set_stream(got)
    a = d.decode_stream(idx[:1700].tolist(), tab, lens, offs)
    b = d.decode_stream(idx[1700:].tolist(), tab, lens, offs)        # stateful across calls
    assert a + b == sym.tolist()
    od = oa.RansDecoder()
    od.set_stream(got)
    assert od.decode_stream(idx.tolist(), tab, lens, offs) == sym.tolist()


def test_rans_empty_and_errors():
    from rgbac.ans import BufferedRansEncoder, RansDecoder
    tab, lens, offs = [[0, 65535, 65536]], [3], [0]
    enc = BufferedRansEncoder()
    assert enc.flush() == oa.BufferedRansEncoder().flush()
    with pytest.raises(RuntimeError, match="CDF index out of range"):
        enc.encode_with_indexes([0], [3], tab, lens, offs)
    assert enc.flush() == oa.BufferedRansEncoder().flush()   # failed put left no records
    d = RansDecoder()
    with pytest.raises(RuntimeError, match="multiple of 4"):
        d.set_stream(b"\x00" * 6)
    s = enc.flush()
    d.set_stream(s)
    with pytest.raises(RuntimeError, match="past the end"):
        d.decode_stream([0] * 64, [[0, 1, 65536]], [3], [0])


def test_gaussian_conditional_tables_match_oracle():
    from rgbac.entropy import GaussianConditional
    from rgbac.models.AutoEncoderRGB_Journal import get_scale_table
    gc = GaussianConditional(None)
    assert gc.update_scale_table(get_scale_table())
    assert not gc.update_scale_table(get_scale_table())          # no force: unchanged
    cdf, lens, offs = oa.gc_update(get_scale_table())
    assert torch.equal(gc.quantized_cdf, cdf)
    assert torch.equal(gc.cdf_length.int(), lens) and torch.equal(gc.offset.int(), offs)
    mult = -oa.standardized_quantile(1e-9 / 2)                   # 6.1094
    center = int(torch.ceil(torch.tensor(256.0) * mult).item())  # 1565
    assert gc.quantized_cdf.shape == (64, 2 * center + 1 + 2)
    # build_indexes vs oracle
    s = torch.exp(torch.empty(2000).uniform_(-4, 6))
    assert torch.equal(gc.build_indexes(s), oa.gc_build_indexes(s, gc.scale_table))


def test_entropy_bottleneck_tables_and_coding_match_oracle():
    from rgbac.entropy import EntropyBottleneck
    torch.manual_seed(3)
    eb = EntropyBottleneck(16)
    with torch.no_grad():
        eb.quantiles.add_(torch.randn_like(eb.quantiles) * 0.7)
    assert eb.update()
    sd = {f"entropy_bottleneck.{k}": v for k, v in eb.state_dict().items()}
    sd.update({f"entropy_bottleneck.{k}": v for k, v in eb.named_parameters()})
    cdf, lens, offs = oa.eb_update(sd)
    assert torch.equal(eb.quantized_cdf, cdf)
    assert torch.equal(eb.cdf_length.int(), lens) and torch.equal(eb.offset.int(), offs)
    z = torch.randn(2, 16, 3, 5) * 6
    strings = eb.compress(z)
    med = eb._get_medians().detach().reshape(1, -1, 1, 1)
    sym = torch.round(z - med).int()
    idx = torch.arange(16).view(16, 1).expand(16, 15).reshape(-1).tolist()
    tab = eb.quantized_cdf.tolist()
    for b in range(2):
        o = oa.BufferedRansEncoder()
        o.encode_with_indexes(sym[b].reshape(-1).tolist(), idx, tab, eb.cdf_length.tolist(),
                              eb.offset.tolist())
        assert strings[b] == o.flush()
    zh = eb.decompress(strings, z.shape[2:])
    assert torch.equal(zh, sym.float() + med)


def test_model_update_builds_every_table():
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder
    net = AutoEncoder()
    assert net.update()
    assert net.gaussian_conditional.quantized_cdf.shape[0] == 64
    assert net.entropy_bottleneck.quantized_cdf.shape[0] == 192
    assert not net.update()
    sd = net.state_dict()
    net2 = AutoEncoder()
    net2.load_state_dict(sd)                                     # CDF buffers resized
    assert torch.equal(net2.entropy_bottleneck.quantized_cdf, net.entropy_bottleneck.quantized_cdf)

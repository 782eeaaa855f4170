"""GPU parity: the HIP path (through the C ABI) against the oracle and the reference's goldens.

Bit-exact throughout (integer/byte work). Sizes the oracle finishes in seconds are compared
stage by stage; the full-size configs are compared record by record against manifests the
real reference produced (tests/golden/make_golden.py).
"""
import hashlib
import os

import numpy as np
import pytest

import bmh
from bmh import synth
from oracle_ffi import golden_calgary, golden_small, manifest

pytestmark = pytest.mark.gpu


def _edge_inputs():
    rng = np.random.default_rng(7)
    cases = {
        "n1": b"a", "n2_same": b"aa", "n2_diff": b"ab", "n3": b"aba", "banana": b"banana",
        "zeros_64k": bytes(65536), "ff_5000": b"\xff" * 5000,
        "period2": b"ab" * 5000, "period3": b"abc" * 3333, "period7_big": (b"abcdefg" * 40000)[:270001],
        "almost_zeros": bytes(30000) + b"\x01" + bytes(30000),
        "two_runs": b"\x00" * 70000 + b"\x01" * 70000,
        "rand_17": rng.integers(0, 256, 17, dtype=np.uint8).tobytes(),
        "rand_1000": rng.integers(0, 256, 1000, dtype=np.uint8).tobytes(),
        "rand_small_alpha": rng.integers(0, 3, 50000, dtype=np.uint8).tobytes(),
        "rand_binary_300k": rng.integers(0, 2, 300000, dtype=np.uint8).tobytes(),
        "text_repeats": (b"the quick brown fox jumps over the lazy dog. " * 3000),
    }
    return cases


EDGE = _edge_inputs()


@pytest.mark.parametrize("name", sorted(EDGE))
def test_bwt_matches_oracle(ctx, oracle, name):
    data = EDGE[name]
    prim, L = bmh.bwt(data, ctx)
    oprim, oL = oracle.bwt(data)
    assert L == oL
    assert prim == oprim


def test_bwt_tiny_blocks_batched(ctx, oracle):
    """n = 1..40 over 1-3 symbol alphabets, all in one batch: periodic / identical rotations."""
    rng = np.random.default_rng(11)
    blocks = []
    for n in range(1, 41):
        for alpha in (1, 2, 3):
            blocks.append(rng.integers(0, alpha, n, dtype=np.uint8).tobytes())
        blocks.append((b"ab" * n)[:n])
    arrs = [np.frombuffer(b, np.uint8) for b in blocks]
    offs = np.zeros(len(arrs) + 1, np.uint64)
    offs[1:] = np.cumsum([a.size for a in arrs])
    d_in, d_L = ctx.alloc(int(offs[-1])), ctx.alloc(int(offs[-1]))
    d_in.upload(np.concatenate(arrs))
    prim = ctx.bwt_dev(d_in, offs, d_L)
    L = d_L.download()
    for i, b in enumerate(blocks):
        op, oL = oracle.bwt(b)
        assert (int(prim[i]), L[int(offs[i]):int(offs[i + 1])].tobytes()) == (op, oL), (i, b)


def test_bwt_big_degenerate(ctx, oracle):
    """4 MiB of zeros and a 4 MiB period-3 block: MSD no-move passes, then rank doubling."""
    for data in (bytes(1 << 22), (b"xyz" * ((1 << 22) // 3 + 1))[: 1 << 22]):
        prim, L = bmh.bwt(data, ctx)
        op, oL = oracle.bwt(data)
        assert prim == op and L == oL


def test_bwt_batch_mixed_blocks(ctx, oracle):
    blocks = [EDGE[k] for k in sorted(EDGE)]
    arrs = [np.frombuffer(b, np.uint8) for b in blocks]
    offs = np.zeros(len(arrs) + 1, np.uint64)
    offs[1:] = np.cumsum([a.size for a in arrs])
    d_in, d_L = ctx.alloc(int(offs[-1])), ctx.alloc(int(offs[-1]))
    d_in.upload(np.concatenate(arrs))
    prim = ctx.bwt_dev(d_in, offs, d_L)
    L = d_L.download()
    for i, b in enumerate(blocks):
        op, oL = oracle.bwt(b)
        assert int(prim[i]) == op, i
        assert L[int(offs[i]):int(offs[i + 1])].tobytes() == oL, i


@pytest.mark.parametrize("name", ["rand_1000", "text_repeats", "zeros_64k", "rand_binary_300k"])
def test_mtf_and_histogram_match_oracle(ctx, oracle, name):
    data = EDGE[name]
    m = bmh.move_to_front(data, ctx)
    assert m == oracle.mtf(data)
    a = np.frombuffer(data, np.uint8)
    d = ctx.alloc(a.size)
    d.upload(a)
    freq, first = ctx.histogram_dev(d, np.array([0, a.size], np.uint64))
    of, ofi = oracle.histogram(data)
    assert (freq[0] == of).all() and (first[0] == ofi).all()
    # bmh_mtf_dev's own histogram / first-occurrence outputs (of its MTF stream)
    d_m = ctx.alloc(a.size)
    mf, mfi = ctx.mtf_dev(d, np.array([0, a.size], np.uint64), d_m)
    hf, hfi = oracle.histogram(m)
    assert (mf[0] == hf).all() and (mfi[0] == hfi).all()


def test_mtf_dev_histograms_batched(ctx, oracle):
    """h_freq / h_first of bmh_mtf_dev (the histogram + first-occurrence scan of huffman(),
    main.cpp:231-244) for a batch of blocks of mixed size and alphabet, against the oracle."""
    rng = np.random.default_rng(11)
    blocks = [rng.integers(0, 256, 70_000, dtype=np.uint8), rng.integers(0, 3, 5_000, dtype=np.uint8),
              np.frombuffer(b"banana", np.uint8), synth.zipf_text(300_000), np.zeros(9_000, np.uint8)]
    a = np.concatenate(blocks)
    offs = np.cumsum([0] + [b.size for b in blocks]).astype(np.uint64)
    d, d_m = ctx.alloc(a.size), ctx.alloc(a.size)
    d.upload(a)
    freq, first = ctx.mtf_dev(d, offs, d_m)
    m = d_m.download()
    for i, b in enumerate(blocks):
        om = oracle.mtf(b)
        assert m[int(offs[i]):int(offs[i + 1])].tobytes() == om, i
        of, ofi = oracle.histogram(om)
        assert (freq[i] == of).all() and (first[i] == ofi).all(), i


def _fib_stream(nsym: int, seed: int) -> np.ndarray:
    """Symbols 0..nsym-1 with Fibonacci frequencies 1, 1, 2, 3, 5, ... in random order: the
    Huffman tree is a chain, so the rarest symbols get codes nsym-1 bits long."""
    f = [1, 1]
    while len(f) < nsym:
        f.append(f[-1] + f[-2])
    rng = np.random.default_rng(seed)
    vals = rng.permutation(nsym).astype(np.uint8)  # which byte value gets which frequency
    return rng.permutation(np.repeat(vals, f[:nsym]))


@pytest.mark.parametrize("nsym", [12, 34, 38])
def test_pack_dev_long_codes(ctx, oracle, nsym):
    """bmh_histogram_dev + bmh_huffman_build + bmh_pack_dev (encode_with_huffman,
    main.cpp:158-172) on a stream whose longest codes are nsym-1 bits (33 and 37 bits take the
    pack's > 32-bit path): code table and tree equal the oracle's, the payload has the
    reference's length, decodes back to the stream and is zero-padded."""
    s = _fib_stream(nsym, nsym)
    d = ctx.alloc(s.size)
    d.upload(s)
    offs = np.array([0, s.size], np.uint64)
    freq, first = ctx.histogram_dev(d, offs)
    of, ofi = oracle.histogram(s)
    assert (freq[0] == of).all() and (first[0] == ofi).all()
    t = bmh.huffman_build(freq[0], first[0])
    oln, ocode, otree = oracle.huffman_build(of, ofi)
    ln = np.frombuffer(bytes(t.len), np.uint8)
    assert (ln == oln).all() and int(ln.max()) == nsym - 1
    code = np.ctypeslib.as_array(t.code)
    assert (code[oln > 0] == ocode[oln > 0]).all()
    assert t.tree_bytes == otree
    payload, t2 = bmh.huffman(s, ctx)
    bits = int((freq[0] * ln.astype(np.uint64)).sum())
    assert len(payload) == max(1, (bits + 7) // 8) == bmh.payload_bytes(t, freq[0])
    if bits % 8:
        assert payload[-1] & ((1 << (8 - bits % 8)) - 1) == 0
    rec = (np.array([0, s.size, len(otree)], np.uint64).tobytes() + otree + payload)
    assert oracle.decode_to_mtf(rec) == s.tobytes()
    assert bmh.record_to_mtf(rec) == s.tobytes()


def _pack_ref(stream: np.ndarray, ln: np.ndarray, code: np.ndarray) -> bytes:
    """encode_with_huffman (main.cpp:158-172) in numpy: code words MSB-first, zero-padded to
    whole bytes, at least one byte."""
    words = {}
    for v in np.unique(stream):
        l = int(ln[v])
        words[int(v)] = np.array([(int(code[v]) >> (l - 1 - j)) & 1 for j in range(l)], np.uint8)
    bits = np.concatenate([words[int(v)] for v in stream]) if stream.size else np.zeros(0, np.uint8)
    out = np.packbits(bits).tobytes()
    return out if out else b"\x00"


def test_pack_dev_multiblock_windows(ctx):
    """bmh_pack_dev over three blocks at unaligned payload offsets, each with its own table:
    block 0 spans three 4096-symbol chunks (a pack workgroup takes 4 chunks, so its table is
    reloaded inside the workgroup at block 1's first chunk); block 1 is made of the rarest
    symbols of a Fibonacci table (> 16 bits per symbol: the chunk image takes several LDS
    windows, codes over 32 bits); block 2 holds one symbol. Every payload equals the numpy
    packing of the reference's encode_with_huffman (main.cpp:158-172)."""
    rng = np.random.default_rng(11)
    tabs, streams = [], []
    for b, (nsym, n) in enumerate([(24, 9000), (40, 10000), (12, 1)]):
        fib = _fib_stream(nsym, 100 + b)
        d = ctx.alloc(fib.size)
        d.upload(fib)
        freq, first = ctx.histogram_dev(d, np.array([0, fib.size], np.uint64))
        d.free()
        t = bmh.huffman_build(freq[0], first[0])
        ln = np.frombuffer(bytes(t.len), np.uint8)
        present = np.flatnonzero(ln)
        if b == 1:  # the ten rarest symbols (codes of 30-39 bits)
            present = present[np.argsort(ln[present])[-10:]]
        streams.append(rng.choice(present, n).astype(np.uint8))
        tabs.append(t)
    refs = [_pack_ref(s, np.frombuffer(bytes(t.len), np.uint8), np.ctypeslib.as_array(t.code))
            for s, t in zip(streams, tabs)]
    assert len(refs[1]) * 8 > 16 * streams[1].size
    po = np.zeros(3, np.uint64)
    po[0] = 3
    po[1] = po[0] + len(refs[0]) + 1
    po[2] = po[1] + len(refs[1]) + 5
    total = int(po[2]) + len(refs[2]) + 8
    allm = np.concatenate(streams)
    offs = np.array([0, streams[0].size, streams[0].size + streams[1].size, allm.size], np.uint64)
    d_m = ctx.alloc(allm.size)
    d_m.upload(allm)
    d_out = ctx.alloc(total)
    d_out.upload(np.full(total, 0xA5, np.uint8))
    ct = (bmh.CodeTable * 3)(*tabs)
    nbytes = np.zeros(3, np.uint64)
    bmh._check(bmh.lib().bmh_pack_dev(ctx.h, d_m.ptr, bmh._u64p(offs), 3, ct, d_out.ptr, total, bmh._u64p(po),
                                      bmh._u64p(nbytes)), "pack")
    out = d_out.download(total).tobytes()
    assert [int(x) for x in nbytes] == [len(r) for r in refs]
    for b in range(3):
        assert out[int(po[b]):int(po[b]) + len(refs[b])] == refs[b], f"block {b}"
    # bytes outside the payloads are untouched (edge words are updated under a mask)
    assert out[:3] == b"\xa5" * 3
    assert out[int(po[0]) + len(refs[0]):int(po[1])] == b"\xa5"

    # pay_offs = NULL: payloads back to back from d_out
    packed = sum(len(r) for r in refs)
    d_out.upload(np.full(total, 0xA5, np.uint8))
    bmh._check(bmh.lib().bmh_pack_dev(ctx.h, d_m.ptr, bmh._u64p(offs), 3, ct, d_out.ptr, (packed + 3) & ~3, None,
                                      None), "pack back to back")
    assert d_out.download(packed).tobytes() == b"".join(refs)

    # the boundary checks its buffer: a payload past out_cap (also by the
    # word-rounded end) is BMH_ERANGE and nothing is written; overlapping payloads are BMH_EINVAL
    d_out.upload(np.full(total, 0xA5, np.uint8))
    L = bmh.lib()
    end2 = int(po[2]) + len(refs[2])
    word_end = (end2 + 3) & ~3
    for cap in (end2 - 1, word_end - 1, 0):
        st = L.bmh_pack_dev(ctx.h, d_m.ptr, bmh._u64p(offs), 3, ct, d_out.ptr, cap, bmh._u64p(po), None)
        assert st == bmh.BMH_ERANGE, cap
    po_bad = po.copy()
    po_bad[1] = po[0] + len(refs[0]) - 1
    st = L.bmh_pack_dev(ctx.h, d_m.ptr, bmh._u64p(offs), 3, ct, d_out.ptr, total, bmh._u64p(po_bad), None)
    assert st == bmh.BMH_EINVAL
    assert d_out.download(total).tobytes() == b"\xa5" * total
    # the context stays usable
    bmh._check(L.bmh_pack_dev(ctx.h, d_m.ptr, bmh._u64p(offs), 3, ct, d_out.ptr, total, bmh._u64p(po), None), "pack")
    assert d_out.download(total).tobytes()[int(po[1]):int(po[1]) + len(refs[1])] == refs[1]
    d_m.free()
    d_out.free()


def test_mtf_long_block_chunked(ctx, oracle):
    # > 64 K symbols per block: exercises the chunk recency / composition path
    rng = np.random.default_rng(3)
    a = np.concatenate([rng.integers(0, 256, 400000, dtype=np.uint8),
                        rng.integers(0, 5, 400000, dtype=np.uint8)])
    assert bmh.move_to_front(a, ctx) == oracle.mtf(a)


def test_calgary_whole_file_records(ctx):
    names, datas, recs = zip(*golden_calgary())
    out = ctx.encode_blocks(datas)
    for n, o, r in zip(names, out, recs):
        assert o == r, n


def test_small_records(ctx):
    for name, data, rec in golden_small():
        assert ctx.encode_blocks([data])[0] == rec, name


def test_records_decode(ctx, oracle):
    for name in ["banana", "period3", "rand_small_alpha", "zeros_64k", "two_runs"]:
        rec = ctx.encode_blocks([EDGE[name]])[0]
        assert bmh.decompress_bytes(rec) == EDGE[name]
        assert oracle.decode(rec) == EDGE[name]


def _blocks_vs_manifest(ctx, man, gen):
    blocks = man["blocks"]
    nb = len(blocks)
    agg = hashlib.sha256()
    step = 64
    for s in range(0, nb, step):
        datas = [gen(b) for b in range(s, min(nb, s + step))]
        outs = ctx.encode_blocks(datas)
        for i, o in enumerate(outs):
            e = blocks[s + i]
            assert len(o) == e["record_len"], (s + i, len(o), e)
            assert int.from_bytes(o[:8], "little") == e["primary"], s + i
            assert hashlib.sha256(o).hexdigest() == e["sha256"], s + i
            agg.update(o)
    assert agg.hexdigest() == man["aggregate_sha256"]


def test_calgary_256k_manifest(ctx):
    man = manifest("calgary_256k")
    blocks = []
    for _, data, _ in golden_calgary():
        for i in range(0, len(data), 262144):
            blocks.append(data[i:i + 262144])
    _blocks_vs_manifest(ctx, man, lambda b: blocks[b])


def test_random_1g_4m_manifest(ctx):
    man = manifest("random_1g_4m")
    _blocks_vs_manifest(ctx, man, lambda b: synth.splitmix64_bytes(0, b << 22, 1 << 22))


def test_zipf_16m_manifest(ctx):
    """Config 5's first 8 blocks as one device batch (the full 512 are streamed below)."""
    man = dict(manifest("zipf_16m"))
    man["blocks"] = man["blocks"][:8]
    z = synth.zipf_text(8 * (16 << 20))
    outs = ctx.encode_blocks([z[b * (16 << 20):(b + 1) * (16 << 20)] for b in range(8)])
    for b, o in enumerate(outs):
        assert hashlib.sha256(o).hexdigest() == man["blocks"][b]["sha256"], b


def test_device_zipf_matches_oracle(ctx, oracle):
    """bmh_synth_zipf_dev (synth.hip) against SURVEY App. D's sha256 of the first 16 MiB and the
    oracle's sequential generator at windows that start and end inside tokens, inside a round and
    across the 2^26-token round boundary (~470 MB)."""
    from oracle_ffi import ZipfStream
    d = ctx.alloc(16 << 20)
    ctx.synth_zipf(d, 16 << 20, 0)
    assert hashlib.sha256(d.download().tobytes()).hexdigest() == \
        "b8b5a2980d7a3c0ec97b8eafa08eaf2423aa1696be1fb47b191566c737d2b889"
    zs = ZipfStream(oracle)
    pos = 0
    for off, n in [(3, 1), (12345, 1000001), (469_999_000, 2_000_000), (512 << 20, 4096)]:
        zs.read(off - pos)
        ref = zs.read(n)
        pos = off + n
        ctx.synth_zipf(d, n, off)
        assert d.download(n).tobytes() == ref.tobytes(), (off, n)


@pytest.mark.timeout(900)
def test_config5_8g_stream_manifest(ctx):
    """BASELINE config 5 on its true input: the 8 GiB App. D Zipf stream (generated in HBM by
    bmh_synth_zipf_dev, copied to pageable host memory), encoded in 16 MiB blocks by
    bmh_compress_host (H2D / encode / D2H overlapped on side streams). All 512 records equal the
    reference's (manifest made by oracle/_ref/ref_COMPRESS, tests/golden/make_golden.py), the
    aggregate sha256 too, and sampled records decode back on the GPU."""
    L = bmh.lib()
    man = manifest("zipf_16m")
    nb = len(man["blocks"])
    assert nb == 512
    bs = 16 << 20
    n = nb * bs
    data = np.empty(n, np.uint8)
    piece = 1 << 30
    d = ctx.alloc(piece)
    for off in range(0, n, piece):
        ctx.synth_zipf(d, piece, off)
        bmh._check(L.bmh_memcpy_d2h(ctx.h, bmh._ptr(data[off:off + piece]), d.ptr, piece), "d2h")
    d.free()
    assert hashlib.sha256(data[:bs]).hexdigest() == \
        "b8b5a2980d7a3c0ec97b8eafa08eaf2423aa1696be1fb47b191566c737d2b889"
    out = np.empty(int(L.bmh_compress_bound(n, bs)), np.uint8)
    olen = ctx.compress_into(data, bs, out)
    assert bmh.is_container(out[:olen])
    hdr = out[:32].view("<u8")
    assert int(hdr[1]) == bs and int(hdr[2]) == nb and int(hdr[3]) == n
    rlen = out[32:32 + 8 * nb].view("<u8").astype(np.int64)
    assert [int(x) for x in rlen] == [b["record_len"] for b in man["blocks"]]
    pos = 32 + 8 * nb
    agg = hashlib.sha256()
    bad = []
    for b in range(nb):
        r = out[pos:pos + int(rlen[b])]
        if hashlib.sha256(r).hexdigest() != man["blocks"][b]["sha256"]:
            bad.append(b)
        agg.update(r)
        if b in (0, 1, 255, 511):
            assert ctx.decompress_bytes(r) == data[b * bs:(b + 1) * bs].tobytes(), b
        pos += int(rlen[b])
    assert pos == olen
    assert not bad, f"{len(bad)} records differ from the reference, first {bad[:8]}"
    assert agg.hexdigest() == man["aggregate_sha256"]


def test_zipf100m_1m_manifest(ctx):
    man = manifest("zipf100m_1m")
    z = synth.zipf_text(100_000_000)
    _blocks_vs_manifest(ctx, man, lambda b: z[b << 20:(b + 1) << 20])


@pytest.mark.gpu
def test_zipf100m_1m_one_batch_four_pipelines(ctx):
    """Config 3 as one 100 MB batch of 1 MiB blocks: past the run screen with >= 16 blocks, so it
    runs on four pipelines (the fourth on the D2H stream; capi.cpp stream_count): every record
    equals the reference manifest and the records land back to back in block order."""
    man = manifest("zipf100m_1m")
    z = synth.zipf_text(100_000_000)
    nb = len(man["blocks"])
    outs = ctx.encode_blocks([z[b << 20:(b + 1) << 20] for b in range(nb)])
    agg = hashlib.sha256()
    for b, o in enumerate(outs):
        assert hashlib.sha256(o).hexdigest() == man["blocks"][b]["sha256"], b
        agg.update(o)
    assert agg.hexdigest() == man["aggregate_sha256"]


def test_device_synth_matches_numpy(ctx):
    for off, n in [(0, 1 << 20), (12345, 100001)]:
        d = ctx.alloc(n)
        ctx.synth_splitmix64(d, n, 0, off)
        assert d.download().tobytes() == synth.splitmix64_bytes(0, off, n).tobytes()


def test_container_roundtrip(ctx):
    data = synth.zipf_text(3_000_001).tobytes()
    out = ctx.compress_bytes(data, block_size=1 << 20)
    assert bmh.is_container(out)
    recs = bmh.container_records(out)
    assert len(recs) == 3
    assert bmh.decompress_bytes(out) == data
    one = ctx.encode_blocks([data[: 1 << 20]])[0]
    assert recs[0] == one


def test_streamed_host_compress_many_batches(ctx):
    """bmh_compress_host's pipeline (staging slots, side-stream H2D/D2H) over many small
    batches, one and two contexts: the container equals the per-block device records."""
    data = synth.zipf_text(9_000_017).tobytes()
    bs = 1 << 20
    blocks = [data[i:i + bs] for i in range(0, len(data), bs)]
    want = ctx.encode_blocks(blocks)
    other = bmh.Context(0)
    try:
        for batch in (bs, 3 * bs + 5, 1 << 30):  # 9, 3 and 1 batches
            for c in (ctx, other):
                c.set_option("stream_batch", batch)
            out = ctx.compress_bytes(data, block_size=bs)
            assert bmh.container_records(out) == want, batch
            multi = bmh.compress_bytes_multi([ctx, other], data, bs)
            assert multi == out, batch
    finally:
        ctx.set_option("stream_batch", 0)
        other.close()
    assert bmh.decompress_bytes(out) == data


# ------------------------------------------------------------------------ GPU decode
def test_gpu_decode_golden_records(ctx):
    """The reference's own records (Calgary + small known answers) decoded on the GPU."""
    for name, data, rec in list(golden_calgary()) + list(golden_small()):
        assert ctx.decompress_bytes(rec) == data, name


def test_gpu_decode_edge_roundtrips(ctx):
    for name in sorted(EDGE):
        rec = ctx.encode_blocks([EDGE[name]])[0]
        assert ctx.decompress_bytes(rec) == EDGE[name], name


def test_gpu_decode_container_roundtrip(ctx):
    data = synth.zipf_text(5_000_003).tobytes()
    out = ctx.compress_bytes(data, block_size=1 << 20)
    assert ctx.decompress_bytes(out) == data


def test_gpu_decode_random_1g_blocks(ctx):
    # full-size blocks of the bench workload: encode -> GPU decode round trip, 16 x 4 MiB
    bs, nb = 1 << 22, 16
    d_in = ctx.alloc(bs * nb)
    ctx.synth_splitmix64(d_in, bs * nb, 0, 0)
    offs = np.arange(nb + 1, dtype=np.uint64) * np.uint64(bs)
    cap = nb * int(bmh.lib().bmh_record_bound(bs))
    d_rec = ctx.alloc(cap)
    ro = ctx.encode_blocks_dev(d_in, offs, d_rec, cap)
    d_dec = ctx.alloc(bs * nb)
    oo = ctx.decode_blocks_dev(d_rec, ro, d_dec, bs * nb)
    assert (oo == offs).all()
    assert d_dec.download().tobytes() == d_in.download().tobytes()


@pytest.mark.parametrize("alpha", [8, 32, 64, 128])
def test_gpu_decode_equal_length_codes(ctx, alpha):
    """iid bytes over 0..alpha-1: the MTF stream stays in that range and every code word has
    the same length (log2 alpha bits), so a segment decoded from a misaligned start never
    resynchronises. The GPU decode must still restore every block (offset-map fallback),
    alone and in a batch with ordinary blocks, and agree with the host decoder."""
    rng = np.random.default_rng(alpha)
    big = rng.integers(0, alpha, 1 << 20, dtype=np.uint8).tobytes()
    rec = ctx.encode_blocks([big])[0]
    ctx.reset_stats()
    ctx.set_timing(True)
    try:
        assert ctx.decompress_bytes(rec) == big
        assert "dec_huff_map" in ctx.kernel_stats()  # the fix-up rounds alone cannot settle this
    finally:
        ctx.set_timing(False)
    assert bmh.decompress_bytes(rec) == big
    blocks = [rng.integers(0, alpha, n, dtype=np.uint8).tobytes() for n in (300_001, 77_777, 5)]
    blocks.insert(1, synth.zipf_text(200_000).tobytes())
    data = b"".join(blocks)
    out = ctx.compress_bytes(data, block_size=len(blocks[0]))
    assert ctx.decompress_bytes(out) == data


@pytest.mark.parametrize("mutate", ["truncate", "bad_n", "bad_tree_len", "bad_primary", "short_payload"])
def test_gpu_decode_corrupt_records(ctx, mutate):
    """Malformed records (cf. decompress(), main.cpp:327-345, which has no checks) come back
    from the GPU decoder as BMH_ECORRUPT, and the context decodes a good record afterwards."""
    name, data, rec = next(golden_calgary())
    r = bytearray(rec)
    if mutate == "truncate":
        r = r[:100]
    elif mutate == "bad_n":
        r[8:16] = (10 ** 12).to_bytes(8, "little")
    elif mutate == "bad_tree_len":
        r[16:24] = (10 ** 6).to_bytes(8, "little")
    elif mutate == "bad_primary":
        r[0:8] = (len(data) + 5).to_bytes(8, "little")
    else:  # n 10 % larger than the payload holds (passes the header checks): the decode runs dry
        r[8:16] = (len(data) * 11 // 10).to_bytes(8, "little")
    with pytest.raises(bmh.BmhError) as e:
        ctx.decompress_bytes(bytes(r))
    assert e.value.status == 5, (mutate, e.value)  # BMH_ECORRUPT
    assert ctx.decompress_bytes(rec) == data


@pytest.mark.gpu
def test_bwt_calgary_batch_repeatable(ctx, oracle):
    # many deferred tie groups per workgroup: the deferral queues overflow into the lists
    # directly, from lanes of one wave bound for different lists (a race here shows up as a
    # few wrong L bytes in some of the repetitions)
    items = [d for _, d, _ in golden_calgary()]
    arrs = [np.frombuffer(d, np.uint8) for d in items]
    offs = np.zeros(len(arrs) + 1, np.uint64)
    offs[1:] = np.cumsum([a.size for a in arrs])
    ref = [oracle.bwt(d) for d in items]
    d_in, d_L = ctx.alloc(int(offs[-1])), ctx.alloc(int(offs[-1]))
    d_in.upload(np.concatenate(arrs))
    for _ in range(30):
        prim = ctx.bwt_dev(d_in, offs, d_L)
        L = d_L.download()
        for i, (p, rL) in enumerate(ref):
            assert int(prim[i]) == p and L[int(offs[i]):int(offs[i + 1])].tobytes() == rL, i


def _fib_word(n):
    a, b = b"a", b"ab"
    while len(b) < n:
        a, b = b, b + a
    return b[:n]


def _fuzz_blocks(seed, count):
    """Seeded mixed-structure blocks: log-uniform sizes 1..300 K over uniform, small-alphabet,
    periodic-with-mutations, Fibonacci-word (deepest tie chains for rank doubling), run-length
    and Zipf-text generators."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(count):
        n = int(np.exp(rng.uniform(0, np.log(300_000)))) or 1
        kind = i % 6
        if kind == 0:
            b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        elif kind == 1:
            b = rng.integers(0, int(rng.integers(1, 5)), n, dtype=np.uint8).tobytes()
        elif kind == 2:
            p = int(rng.integers(1, 64))
            a = np.resize(rng.integers(0, 256, p, dtype=np.uint8), n)
            if n > 4:
                a[rng.integers(0, n, max(1, n // 5000))] ^= 1
            b = a.tobytes()
        elif kind == 3:
            b = _fib_word(n)
        elif kind == 4:
            runs = rng.integers(1, 2000, n // 8 + 1)
            b = np.repeat(rng.integers(0, 4, runs.size, dtype=np.uint8), runs)[:n].tobytes()
            b = b + bytes(n - len(b))
        else:
            b = synth.zipf_text(n).tobytes()
        out.append(b)
    return out


@pytest.mark.parametrize("seed", [101, 202])
def test_fuzz_batch_bwt_mtf_roundtrip(ctx, oracle, seed):
    """One batch of 48 mixed blocks: BWT (L, primary) and MTF bit-exact against the oracle,
    then encode -> GPU decode restores every block."""
    blocks = _fuzz_blocks(seed, 48)
    arrs = [np.frombuffer(b, np.uint8) for b in blocks]
    offs = np.zeros(len(arrs) + 1, np.uint64)
    offs[1:] = np.cumsum([a.size for a in arrs])
    d_in, d_L = ctx.alloc(int(offs[-1])), ctx.alloc(int(offs[-1]))
    d_in.upload(np.concatenate(arrs))
    prim = ctx.bwt_dev(d_in, offs, d_L)
    L = d_L.download()
    for i, b in enumerate(blocks):
        op, oL = oracle.bwt(b)
        got = L[int(offs[i]):int(offs[i + 1])].tobytes()
        assert int(prim[i]) == op and got == oL, (i, len(b))
        if i % 4 == 0:
            assert bmh.move_to_front(b, ctx) == oracle.mtf(b), (i, len(b))
    recs = ctx.encode_blocks(blocks)
    for i, (b, r) in enumerate(zip(blocks, recs)):
        assert ctx.decompress_bytes(r) == b, (i, len(b))


@pytest.mark.parametrize("kind", ["random_64m", "zipf_64m", "period5_32m"])
def test_large_single_block_roundtrip(ctx, kind):
    """Blocks far past the bench's 4 MiB (the oracle needs over a minute here), checked through
    size-independent properties: record header n, L a permutation of the block, encode
    determinism, and encode -> GPU decode restoring the block."""
    if kind == "random_64m":
        a = np.random.default_rng(5).integers(0, 256, 64 << 20, dtype=np.uint8)
    elif kind == "zipf_64m":
        a = synth.zipf_text(64 << 20)
    else:
        a = np.frombuffer((b"abcde" * ((32 << 20) // 5 + 1))[: 32 << 20], np.uint8)
    data = a.tobytes()
    d_in, d_L = ctx.alloc(a.size), ctx.alloc(a.size)
    d_in.upload(a)
    offs = np.array([0, a.size], np.uint64)
    prim = ctx.bwt_dev(d_in, offs, d_L)
    assert 0 <= int(prim[0]) < a.size
    assert (np.bincount(d_L.download(), minlength=256) == np.bincount(a, minlength=256)).all()
    r1 = ctx.encode_blocks([data])[0]
    r2 = ctx.encode_blocks([data])[0]
    assert r1 == r2
    assert int(np.frombuffer(r1[:24], np.uint64)[1]) == a.size
    assert int(np.frombuffer(r1[:24], np.uint64)[0]) == int(prim[0])
    assert ctx.decompress_bytes(r1) == data


def test_device_errors_are_status_codes(ctx):
    """Empty blocks (the reference segfaults) and short output buffers come back as
    BMH_EINVAL / BMH_ERANGE, and the context stays usable afterwards."""
    with pytest.raises(bmh.BmhError) as e:
        ctx.encode_blocks([b"abc", b""])
    assert e.value.status == 1  # BMH_EINVAL
    a = np.random.default_rng(9).integers(0, 256, 1 << 16, dtype=np.uint8)
    d_in = ctx.alloc(a.size)
    d_in.upload(a)
    d_out = ctx.alloc(1024)
    with pytest.raises(bmh.BmhError) as e:
        ctx.encode_blocks_dev(d_in, np.array([0, a.size], np.uint64), d_out, 1024)
    assert e.value.status == 4  # BMH_ERANGE
    assert ctx.decompress_bytes(ctx.encode_blocks([a.tobytes()])[0]) == a.tobytes()


def test_compress_host_pinned_buffers(ctx):
    """bmh_compress_host with page-locked input and output (bmh_host_alloc: DMA-only path,
    records D2H'd straight to their place) writes the same bytes as with pageable buffers;
    several stream batches, a single block, and a too-small page-locked output (ERANGE)."""
    ctx.set_option("stream_batch", 3 << 20)
    data = np.frombuffer(synth.zipf_text(10_000_019).tobytes(), np.uint8)
    hin = ctx.alloc_host(data.size)
    hin.a[:] = data
    try:
        for bs in (1 << 20, 1 << 24):
            ref = ctx.compress_bytes(data, block_size=bs)
            cap = int(bmh.lib().bmh_compress_bound(data.size, bs))
            hout = ctx.alloc_host(cap)
            n = ctx.compress_into(hin.a, bs, hout.a)
            assert hout.a[:n].tobytes() == ref, bs
            n2 = ctx.compress_into(data, bs, hout.a)  # pageable in, pinned out
            assert hout.a[:n2].tobytes() == ref, bs
            out = np.empty(cap, np.uint8)
            n3 = ctx.compress_into(hin.a, bs, out)  # pinned in, pageable out
            assert out[:n3].tobytes() == ref, bs
            hout.free()
        small = ctx.alloc_host(1000)
        with pytest.raises(bmh.BmhError) as e:
            ctx.compress_into(hin.a, 1 << 20, small.a)
        assert e.value.status == 4  # BMH_ERANGE
        small.free()
        assert ctx.decompress_bytes(ctx.compress_bytes(data[:5000], 0)) == data[:5000].tobytes()
    finally:
        hin.free()
        ctx.set_option("stream_batch", 0)


def test_compress_host_multi_matches_single_context(ctx):
    """bmh_compress_host_multi (one context + host thread each, blocks dealt round-robin)
    assembles the same container as one context; here several contexts share the test GPU.
    Includes more contexts than blocks (a context with nothing to do) and a single block."""
    data = synth.zipf_text(9_000_007).tobytes()
    extra = [bmh.Context(0), bmh.Context(0)]
    try:
        for bs in (1 << 20, 3 << 20, 1 << 24):  # 9, 3 and 1 blocks
            single = ctx.compress_bytes(data, block_size=bs)
            multi = bmh.compress_bytes_multi([ctx] + extra, data, bs)
            assert multi == single, bs
            assert ctx.decompress_bytes(multi) == data, bs
        small = data[:5000]
        assert bmh.compress_bytes_multi([ctx] + extra, small, 4096) == ctx.compress_bytes(small, block_size=4096)
    finally:
        for c in extra:
            c.close()


def test_fresh_context_single_data_phase():
    """a one-shot encode of Calgary's progl (a block whose long repeats need
    rank doubling) on a fresh context runs the BWT data phase once — small batches store the full
    SA from the start instead of re-running the data phase when doubling turns out to be needed —
    and its record is still the reference's. (pic, the first file this held for, now takes the
    run-length path: tests/test_gpu_runs.py.)"""
    from oracle_ffi import GOLDEN
    progl = open(os.path.join(GOLDEN, "calgary", "progl"), "rb").read()
    gold = open(os.path.join(GOLDEN, "calgary_records", "progl.bzap"), "rb").read()
    with bmh.Context(0) as fresh:
        fresh.reset_stats()
        fresh.set_timing(True)
        rec = fresh.encode_blocks([progl])[0]
        st = fresh.kernel_stats()
        fresh.set_timing(False)
    assert rec == gold
    assert st["bwt_g1_scatter"][0] == 1, st.get("bwt_g1_scatter")
    assert st.get("bwt_rank_fill", (0, 0))[0] == 1  # progl does need the doubling phase


def test_compress_host_multi_distinct_devices(ctx):
    """bmh_compress_host_multi with one context on EACH visible GPU (the in-process form of the
    round-robin deal over 1-8 GPUs): same container as one context, with pageable
    and with page-locked input (the pinned fast path must hold for contexts on other devices
    than the one the buffer was registered on). Skipped on a one-GPU box: the shared-device
    case is test_compress_host_multi_matches_single_context."""
    ndev = int(bmh.lib().bmh_device_count())
    if ndev < 2:
        pytest.skip(f"{ndev} GPU visible: distinct-device contexts need >= 2 (the shared-device case runs above)")
    data = synth.zipf_text(9_000_007).tobytes()
    ctxs = [ctx] + [bmh.Context(d) for d in range(1, min(ndev, 8))]
    hin = ctx.alloc_host(len(data))
    hin.a[:] = np.frombuffer(data, np.uint8)
    try:
        for bs in (1 << 20, 3 << 20):
            single = ctx.compress_bytes(data, block_size=bs)
            assert bmh.compress_bytes_multi(ctxs, data, bs) == single, bs
            assert bmh.compress_bytes_multi(ctxs, hin.a, bs) == single, bs
        assert ctx.decompress_bytes(single) == data
    finally:
        hin.free()
        for c in ctxs[1:]:
            c.close()


def test_cli_compress_matches_reference_binary(tmp_path):
    """`bmh_compress <in> <out>` (the reference's COMPRESS binary, main.cpp:439-447) on the GPU:
    every Calgary record byte-identical to the reference's and its stdout line the same;
    `bmh decompress` restores the file."""
    import json
    import os
    import subprocess
    from oracle_ffi import GOLDEN
    cli = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "bwt-mtf-huffman-compressor_amd", "bin", "bmh")
    assert os.path.exists(cli), "CLI not built"
    gold = {e["file"]: e["stdout_tail"] for e in json.load(open(os.path.join(GOLDEN, "calgary_stdout.json")))}
    for name, data, rec in golden_calgary():
        src, dst, back = tmp_path / name, tmp_path / (name + ".bzap"), tmp_path / (name + ".out")
        src.write_bytes(data)
        r = subprocess.run([cli + "_compress", str(src), str(dst)], capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr
        assert dst.read_bytes() == rec, name
        assert r.stdout.endswith(gold[name]), (name, r.stdout)
        r = subprocess.run([cli, "decompress", str(dst), str(back)], capture_output=True, text=True, timeout=60)
        assert r.returncode == 0 and back.read_bytes() == data, name


def test_cli_full_pipeline_calgary(tmp_path):
    """`bmh_full_pipeline` run like the reference's FULL_PIPELINE binary (main.cpp:416-438: no
    arguments, ./calgarycorpus/): stdout is byte-identical to the reference's (the `k/14 `
    prefixes, compress lines and `success` verdicts; tests/golden/full_pipeline/stdout.txt),
    every .decoded file equals its input, and every .bzap has the size of the reference's
    FULL_PIPELINE record. Their bytes equal the reference's standalone COMPRESS records: the
    reference's FULL_PIPELINE tree bytes also depend on heap history carried over from the
    previous files (13 of 14 differ), which bmh does not model; the reference's
    decoder reads both."""
    import os
    import shutil
    import subprocess
    from oracle_ffi import GOLDEN, REF_DIR
    cli = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "bwt-mtf-huffman-compressor_amd", "bin", "bmh")
    d = tmp_path / "calgarycorpus"
    shutil.copytree(os.path.join(GOLDEN, "calgary"), d)
    r = subprocess.run([cli + "_full_pipeline"], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    fp = os.path.join(GOLDEN, "full_pipeline")
    assert r.stdout == open(os.path.join(fp, "stdout.txt")).read()
    recs = {name: rec for name, _, rec in golden_calgary()}
    for name in recs:
        out = (d / (name + ".bzap")).read_bytes()
        assert len(out) == os.path.getsize(os.path.join(fp, name + ".bzap")), name
        assert out == recs[name], name
        assert (d / (name + ".decoded")).read_bytes() == (d / name).read_bytes(), name
    dec = os.path.join(REF_DIR, "ref_DECOMPRESS")
    if os.path.exists(dec):  # the reference decoder reads our records
        for name in ("bib", "pic", "trans"):
            subprocess.run([dec, f"calgarycorpus/{name}.bzap", f"{name}.ref"], cwd=tmp_path, check=True,
                           capture_output=True, timeout=120)
            assert (tmp_path / f"{name}.ref").read_bytes() == (d / name).read_bytes(), name


@pytest.mark.gpu
def test_checked_build_full_exec():
    """the checked library (`make check`, -DBMH_CHECK) counts every call of a
    full-wave primitive (DPP wave scan, one-barrier workgroup scan) made with a partial EXEC
    mask. tests/check_workload.py drives every kernel family through it (Calgary records vs the
    reference, tiny / ragged / periodic / binary / Zipf / random blocks, GPU decode round
    trips) and must see identical results and zero violations."""
    import json
    import subprocess
    import sys
    # the in-tree checked build, whatever library BMH_LIB points the rest of the suite at
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    chk = os.path.join(repo, "bwt-mtf-huffman-compressor_amd", "lib_check", "libbmh.so")
    assert os.path.exists(chk), "lib_check/libbmh.so not built (make -C bwt-mtf-huffman-compressor_amd check)"
    env = dict(os.environ, BMH_LIB=os.path.abspath(chk))
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "check_workload.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res == {"mismatches": 0, "exec_violations": 0}, res


def _alpha_block(rng, n, k, kind):
    """n bytes over k distinct values (spread over 0..255), as random draws or runs of words."""
    vals = np.sort(rng.choice(256, k, replace=False)).astype(np.uint8)
    if kind == "uniform":
        idx = rng.integers(0, k, n)
    elif kind == "repeats":  # slices of one base text: ties tens to hundreds of symbols deep
        base = rng.integers(0, k, 6000)
        parts, tot = [], 0
        while tot < n:
            a = int(rng.integers(0, 5600))
            parts.append(base[a:a + int(rng.integers(40, 400))])
            tot += parts[-1].size
        idx = np.concatenate(parts)[:n]
    else:  # Zipf-like words: repeated short patterns
        words = [rng.integers(0, k, int(rng.integers(2, 9))) for _ in range(50)]
        seq, tot = [], 0
        while tot < n:
            w = words[min(int(rng.zipf(1.3)) - 1, 49)]
            seq.append(w)
            tot += w.size
        idx = np.concatenate(seq)[:n]
    return vals[idx].tobytes()


def test_compacted_alphabet_global_pass(ctx, oracle):
    """blocks of k <= 32 distinct bytes key the global pass on s whole symbols
    (s = 3 for k <= 10, 2 for k <= 32; ranks among the block's bytes, db = 8 s) instead of 10 raw
    bits (only the global pass uses the compacted digits; the record and every later pass stay on
    raw rotation bits). Boundary
    alphabets (1, 2, 10, 11, 32, 33 distinct bytes), tiny blocks, uniform, word-like and
    deep-repeat text, values spread over the byte range, all in one batch past the run screen's
    batch size (so no block takes the run path): BWT and records equal the oracle's."""
    rng = np.random.default_rng(2024)
    blocks, rec_check = [], []
    for k in (1, 2, 3, 4, 10, 11, 26, 27, 32, 33):
        for n in (1, 2, 3, 17, 5000, 300_001):
            blocks.append(_alpha_block(rng, n, k, "uniform" if n % 2 else "words"))
        rec_check.append(len(blocks) - 1)
        if k >= 3:
            blocks.append(_alpha_block(rng, 1 << 20, k, "words"))
            rec_check.append(len(blocks) - 1)
        # deep ties: the list rounds' compacted windows (w = 1 .. 5 bits a symbol, 12 .. 16
        # symbols a window, partial-byte starts from the dense finish's deferrals)
        blocks.append(_alpha_block(rng, 200_003, k, "repeats"))
        rec_check.append(len(blocks) - 1)
    blocks.append(synth.zipf_text(3 << 20).tobytes())
    rec_check.append(len(blocks) - 1)
    pad = synth.splitmix64_bytes(0, 0, 70 << 20).tobytes()  # a random block: the batch is past the run screen
    allb = blocks + [pad]
    offs = np.zeros(len(allb) + 1, np.uint64)
    offs[1:] = np.cumsum([len(b) for b in allb])
    d_in, d_L = ctx.alloc(int(offs[-1])), ctx.alloc(int(offs[-1]))
    d_in.upload(np.frombuffer(b"".join(allb), np.uint8))
    prim = ctx.bwt_dev(d_in, offs, d_L)
    L = d_L.download()
    d_in.free()
    d_L.free()
    for i, b in enumerate(blocks):
        op, oL = oracle.bwt(b)
        assert int(prim[i]) == op and L[int(offs[i]):int(offs[i + 1])].tobytes() == oL, (i, len(b), len(set(b)))
    recs = ctx.encode_blocks(allb)
    for i in rec_check:
        assert recs[i] == oracle.encode(blocks[i]), (i, len(blocks[i]))


def test_tuning_options_never_change_records(ctx, oracle):
    """Every non-default bmh_ctx_set_option value (include/bmh.h BMH_OPT_*) once: pipelines 1..4
    and 5, MTF chunks 64 / 1024 / 4096, the list-round checker, and small stream / max batches on
    the host-buffer path, against the default encode of a mixed batch (random, Zipf text, a
    run-heavy block, tiny blocks). Unknown options and out-of-range values are status codes."""
    rng = np.random.default_rng(5)
    blocks = [rng.integers(0, 256, 1 << 20, dtype=np.uint8).tobytes() for _ in range(6)]
    z = synth.zipf_text(6 << 20).tobytes()
    blocks += [z[i:i + (1 << 20)] for i in range(0, len(z), 1 << 20)]
    blocks += [bytes(200000) + b"\x01" * 100000, b"banana", b"a" * 40, rng.integers(0, 4, 70000, np.uint8).tobytes()]
    want = ctx.encode_blocks(blocks)
    for i in (0, 6, 12, 15):  # the default's short MTF chunks take the five-level composition
        assert want[i] == oracle.encode(blocks[i]), i
    try:
        for name, vals in (("pipelines", (1, 2, 3, 4, 5)), ("mtf_chunk", (64, 1024, 4096)), ("check_lists", (1,)), ("one_pipeline", (1,))):
            for v in vals:
                ctx.set_option(name, v)
                assert ctx.encode_blocks(blocks) == want, (name, v)
            ctx.set_option(name, 0)
        data = b"".join(blocks[:12])
        ref = ctx.compress_bytes(data, block_size=1 << 20)
        for name, v in (("stream_batch", 3 << 20), ("max_batch", 2 << 20), ("copy_threads", 2)):
            ctx.set_option(name, v)
            assert ctx.compress_bytes(data, block_size=1 << 20) == ref, name
            assert ctx.decompress_bytes(ref) == data, name
            ctx.set_option(name, 0)
    finally:
        for name in bmh.Context.OPTIONS:
            ctx.set_option(name, 0)
    for opt, v, st in ((99, 1, 1), (1, 17, 4), (4, 5000, 4), (4, 10, 4), (7, 65, 4)):
        assert bmh.lib().bmh_ctx_set_option(ctx.h, opt, v) == st, (opt, v)


def test_dense_probe_pipelines(ctx):
    """encode_blocks' digram census (bwt_runs.hip dense_batch): a 48 MiB batch of random 4 MiB
    blocks runs on one pipeline, the same size of Zipf text on the size rule's three; records
    are the reference's either way (random blocks 0..11 of the config-4 manifest)."""
    bs, nblk = 4 << 20, 12
    offs = np.arange(nblk + 1, dtype=np.uint64) * np.uint64(bs)
    d_in = ctx.alloc(bs * nblk)
    for i in range(nblk):
        ctx.synth_splitmix64(d_in.ptr.value + i * bs, bs, 0, i * bs)
    cap = nblk * int(bmh.lib().bmh_record_bound(bs))
    d_out = ctx.alloc(cap)
    ro = ctx.encode_blocks_dev(d_in, offs, d_out, cap)
    assert ctx.last_pipelines() == 1
    assert ctx.pipelines(bs * nblk, nblk) == 3
    # past 64 MiB: four pipelines from 8 blocks on (128 MB of Zipf in 8 x 16 MiB blocks), two below
    assert ctx.pipelines(128 << 20, 8) == 4 and ctx.pipelines(128 << 20, 7) == 2
    man = manifest("random_1g_4m")["blocks"]
    recs = d_out.download(int(ro[-1])).tobytes()
    for b in range(nblk):
        assert hashlib.sha256(recs[int(ro[b]):int(ro[b + 1])]).hexdigest() == man[b]["sha256"], b
    z = synth.zipf_text(bs * nblk)
    d_in.upload(z)
    ctx.encode_blocks_dev(d_in, offs, d_out, cap)
    assert ctx.last_pipelines() == 3
    ctx.set_option("pipelines", 2)
    ctx.encode_blocks_dev(d_in, offs, d_out, cap)
    assert ctx.last_pipelines() == 2
    ctx.set_option("pipelines", 0)


def test_speculative_list_round_fallback(ctx, oracle):
    """Dense one-pipeline batches run their tiny list round without the host wait and check its
    counters at the end (bwt.hip bwt_spec_ok): a 48 MiB random batch needs no fallback (records
    = the config-4 manifest's); the same batch with a 2 KB stretch of block 5 repeated inside the
    block (rotations tied for up to 16 K bits: more list rounds, then rank doubling) falls back
    once and its records equal the reference's; then a clean batch speculates again; then 400 tied
    pairs in one lane (past the speculative grid) fall back once more."""
    bs, nblk = 4 << 20, 12
    offs = np.arange(nblk + 1, dtype=np.uint64) * np.uint64(bs)
    d_in = ctx.alloc(bs * nblk)
    for i in range(nblk):
        ctx.synth_splitmix64(d_in.ptr.value + i * bs, bs, 0, i * bs)
    cap = nblk * int(bmh.lib().bmh_record_bound(bs))
    d_out = ctx.alloc(cap)
    man = manifest("random_1g_4m")["blocks"]

    def run():
        ro = ctx.encode_blocks_dev(d_in, offs, d_out, cap)
        assert ctx.last_pipelines() == 1
        recs = d_out.download(int(ro[-1])).tobytes()
        return [recs[int(ro[b]):int(ro[b + 1])] for b in range(nblk)]

    f0 = ctx.spec_fallbacks()
    recs = run()
    assert ctx.spec_fallbacks() == f0
    for b in range(nblk):
        assert hashlib.sha256(recs[b]).hexdigest() == man[b]["sha256"], b
    blk = bytearray(synth.splitmix64_bytes(0, 5 * bs, bs).tobytes())
    blk[2_000_000:2_002_048] = blk[1000:3048]
    d_in.upload(np.frombuffer(bytes(blk), np.uint8), offset=5 * bs)
    recs = run()
    assert ctx.spec_fallbacks() == f0 + 1
    assert recs[5] == oracle.encode(bytes(blk))
    for b in (0, 4, 6, 11):
        assert hashlib.sha256(recs[b]).hexdigest() == man[b]["sha256"], b
    ctx.synth_splitmix64(d_in.ptr.value + 5 * bs, bs, 0, 5 * bs)
    recs = run()
    assert ctx.spec_fallbacks() == f0 + 1
    assert hashlib.sha256(recs[5]).hexdigest() == man[5]["sha256"]
    # more tied pairs in one XCD lane than the speculative grid covers (256 entries): 400
    # 12-byte copies in block 5 (each pair resolved in the one tiny round) -> one fallback
    blk = bytearray(synth.splitmix64_bytes(0, 5 * bs, bs).tobytes())
    rng = np.random.default_rng(3)
    for src in rng.choice(np.arange(0, bs // 2 - 64, 64), 400, replace=False):
        dst = int(src) + bs // 2
        blk[dst:dst + 12] = blk[int(src):int(src) + 12]
    d_in.upload(np.frombuffer(bytes(blk), np.uint8), offset=5 * bs)
    recs = run()
    assert ctx.spec_fallbacks() == f0 + 2
    assert recs[5] == oracle.encode(bytes(blk))


def test_planted_ties_in_large_batch(ctx, oracle):
    """Tied rotations in a 20 MiB batch (past the full-SA size, so the dense finish stores SA
    only for segments a later pass reads): three config-4 random blocks (records equal the
    reference manifest), a random block with planted ties — rotation 0's first 8 bytes copied to
    three places (two in its own 16 K chunk), so rotation 0 sits in a tied group whose primary
    the list pass sets; and a 3-byte pattern at 120 places, so one 12-bit sub-bucket holds > 64
    rotations (a digit-level deferral) — and a random block of period 1000 (every rotation tied
    far past 512 bits: the block needs rank doubling and the data phase re-runs with the full
    suffix array). BWT of the crafted blocks equals the oracle's, and all records decode back.
    (Written for the 6-byte record experiment of DESIGN §15, kept for the tie paths.)"""
    bs = 4 << 20
    rng = np.random.default_rng(77)
    blocks = [synth.splitmix64_bytes(0, i * bs, bs).tobytes() for i in range(3)]
    a = rng.integers(0, 256, bs, dtype=np.uint8)
    for at in (1000, 5000, 3_000_000):
        a[at:at + 8] = a[0:8]
    pat = np.array([0x5A, 0xC3, 0x17], np.uint8)
    for at in rng.choice(bs - 3, 120, replace=False):
        a[at:at + 3] = pat
    blocks.append(a.tobytes())
    per = rng.integers(0, 256, 1000, dtype=np.uint8)
    blocks.append(np.tile(per, bs // 1000 + 1)[:bs].tobytes())
    recs = ctx.encode_blocks(blocks)
    man = manifest("random_1g_4m")["blocks"]
    for i in range(3):
        assert hashlib.sha256(recs[i]).hexdigest() == man[i]["sha256"], i
    for i in (3, 4):
        prim, L = bmh.bwt(blocks[i], ctx)
        oprim, oL = oracle.bwt(blocks[i])
        assert prim == oprim and L == oL, i
    for r, d in zip(recs, blocks):
        assert ctx.decompress_bytes(r) == d


def test_tied_pairs_across_windows(ctx, oracle):
    """Tied pairs whose shared prefix ends inside each of the first windows the tiny list pass
    looks at (it extends a tied pair up to 4 windows of 64 bits before deferring it): a random
    1 MiB block with substrings of 9..80 bytes copied once each, one copied across the block end
    (the rotation wraps), plus small blocks whose rotations all tie to the final depth (period
    n / 2). BWT equals the oracle's and every record decodes back."""
    rng = np.random.default_rng(2025)
    bs = 1 << 20
    a = rng.integers(0, 256, bs, dtype=np.uint8)
    at = 4096
    for ln in (9, 15, 16, 17, 24, 31, 32, 33, 40, 41, 48, 56, 63, 64, 65, 72, 80):
        src = int(rng.integers(0, bs - 100))
        a[at:at + ln] = a[src:src + ln]
        at += 3000
    a[bs - 20:] = a[500:520]  # the rotation at bs - 20 matches 20 bytes, then wraps to a[0:]
    a[0:30] = a[520:550]
    per = rng.integers(0, 256, 50, dtype=np.uint8)
    blocks = [a.tobytes(), np.tile(per, 2).tobytes(), np.tile(per[:7], 2).tobytes(),
              rng.integers(0, 4, 300, dtype=np.uint8).tobytes()]
    for blk in blocks:
        prim, L = bmh.bwt(blk, ctx)
        oprim, oL = oracle.bwt(blk)
        assert prim == oprim and L == oL, len(blk)
    for r, d in zip(ctx.encode_blocks(blocks), blocks):
        assert ctx.decompress_bytes(r) == d


def test_speculative_round_with_run_heavy_block(ctx, oracle):
    """A dense batch (11 random 4 MiB blocks) that also holds a 1 MiB run-heavy block (runs of
    4..12 bytes: <= n / 4 runs): one pipeline with the speculative list round for the sorter
    blocks, while the screen sends the run-heavy block to the run path on the side stream; no
    fallback, every record the reference's."""
    bs, nr = 4 << 20, 11
    rng = np.random.default_rng(31)
    vals = rng.integers(0, 256, 200000, dtype=np.uint8)
    lens = rng.integers(4, 13, 200000)
    run_blk = np.repeat(vals, lens)[: 1 << 20].tobytes()
    sizes = [bs] * 5 + [len(run_blk)] + [bs] * 6
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    d_in = ctx.alloc(int(offs[-1]))
    g = 0
    for i, n in enumerate(sizes):
        if i == 5:
            d_in.upload(np.frombuffer(run_blk, np.uint8), offset=int(offs[i]))
        else:
            ctx.synth_splitmix64(d_in.ptr.value + int(offs[i]), bs, 0, g * bs)
            g += 1
    cap = sum(int(bmh.lib().bmh_record_bound(n)) for n in sizes)
    d_out = ctx.alloc(cap)
    f0 = ctx.spec_fallbacks()
    ro = ctx.encode_blocks_dev(d_in, offs, d_out, cap)
    assert ctx.last_pipelines() == 1 and ctx.spec_fallbacks() == f0
    recs = d_out.download(int(ro[-1])).tobytes()
    man = manifest("random_1g_4m")["blocks"]
    g = 0
    for i in range(len(sizes)):
        r = recs[int(ro[i]):int(ro[i + 1])]
        if i == 5:
            assert r == oracle.encode(run_blk)
        else:
            assert hashlib.sha256(r).hexdigest() == man[g]["sha256"], i
            g += 1


def _hip_free_bytes() -> int:
    """Free device memory by hipMemGetInfo of the HIP runtime libbmh runs on: the process's
    libamdhip64 (ROCm's, or torch's copy when torch loaded first and libbmh's dependency resolved
    to it; ROCm's when both are mapped)."""
    import ctypes as C
    bmh.lib()
    paths = [ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64.so" in ln]
    assert paths, "no HIP runtime mapped"
    path = next((p for p in paths if "torch" not in p), paths[0])
    hip = C.CDLL(path)
    free, total = C.c_size_t(), C.c_size_t()
    assert hip.hipMemGetInfo(C.byref(free), C.byref(total)) == 0
    return free.value


def test_text_batch_device_memory_stays_flat():
    """a 128 MiB text batch (not dense: the multi-pipeline path on sub-contexts) must
    not make the parent context also hold the dense prologue's BWT workspaces (~40 bytes per
    input byte), and a second batch of the same layout allocates nothing more."""
    c = bmh.Context(0)  # fresh: no dense batch of this layout before
    n, bs = 128 << 20, 4 << 20
    d_in = c.alloc(n)
    c.synth_zipf(d_in, n, 0)
    offs = np.arange(0, n + 1, bs, dtype=np.uint64)
    cap = int(sum(bmh.lib().bmh_record_bound(bs) for _ in range(n // bs)))
    d_out = c.alloc(cap)
    free0 = _hip_free_bytes()
    ro1 = c.encode_blocks_dev(d_in, offs, d_out, cap)
    assert c.last_pipelines() > 1  # the text path: sub-contexts, not the dense single pipeline
    free1 = _hip_free_bytes()
    ro2 = c.encode_blocks_dev(d_in, offs, d_out, cap)
    free2 = _hip_free_bytes()
    assert np.array_equal(ro1, ro2)
    grew = free0 - free1
    print(f"text batch: {grew / n:.1f} B of device memory per input byte, then {(free1 - free2) >> 20} MiB")
    # the sub-contexts' own workspaces measure ~60 B a byte; the parent's unused dense prologue
    # would add ~40 more
    assert grew <= 72 * n, f"first text batch took {grew / n:.1f} bytes of device memory per input byte"
    assert free1 - free2 <= 64 << 20, f"second batch of the same layout allocated {(free1 - free2) >> 20} MiB"
    del c

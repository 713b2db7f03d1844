"""GPU parity: the HIP codec (through the C ABI) against the reference's
golden vectors and the oracle.  Bit-exact: compressed bytes identical to the
reference encoder, decoded bytes identical, accept/reject identical."""
from __future__ import annotations

import hashlib
import os
import threading

import numpy as np
import pytest

import oracle
from lcdb_amd import corpus

pytestmark = pytest.mark.gpu

# LGS_TEST_PROBE=1 (tests/test_gpu_probe_decoders.py runs this file so in a
# subprocess): the library is the probe build (conftest.py), and the tests
# below also cover the decoders that lost their A/B and exist only there.
PROBE = os.environ.get("LGS_TEST_PROBE") == "1"


def _with_probe(kernels, probe_kernels):
    return list(kernels) + [pytest.param(k, marks=pytest.mark.probe) for k in probe_kernels
                            if PROBE]


def test_dropin_encode_golden(gpu, vectors):
    for v in vectors:
        if v.kind == 0:
            assert gpu.encode(v.a) == v.b, v.name


def test_dropin_decode_golden(gpu, vectors):
    for v in vectors:
        if v.kind == 0:
            assert gpu.decode(v.b) == v.a, v.name
        else:
            out = gpu.decode(v.a)
            assert (out is not None) == bool(v.ok), v.name
            if v.ok:
                assert out == v.b, v.name


def test_dropin_ramp_known_answer(gpu, digests):
    # t-snappy.c:24-53 (1 MiB input: 16 chunks of 64 KiB, one drop-in pass)
    data = bytes(i & 0xFF for i in range(1 << 20))
    enc = gpu.encode(data)
    assert len(enc) == 53203
    assert hashlib.sha256(enc).hexdigest() == digests["ramp_1MiB"]["comp_sha256"]
    assert gpu.decode_size(enc) == 1 << 20
    assert gpu.decode(enc) == data


def test_batch_host_golden(gpu, vectors):
    enc = [v for v in vectors if v.kind == 0 and len(v.a) <= 65536]
    outs = gpu.encode_batch_host([v.a for v in enc])
    for v, o in zip(enc, outs):
        assert o == v.b, v.name
    res, st = gpu.decode_batch_host([v.b for v in enc], [len(v.a) for v in enc])
    for v, o, s in zip(enc, res, st):
        assert s == gpu.LGS_ST_OK and o == v.a, v.name
    dec = [v for v in vectors if v.kind == 1]
    caps = [len(v.b) if v.ok else 4096 for v in dec]
    res, st = gpu.decode_batch_host([v.a for v in dec], caps)
    for v, o, s in zip(dec, res, st):
        if v.ok:
            assert s == gpu.LGS_ST_OK and o == v.b, v.name
        else:
            # a reject may also be reported as "no space" when the bogus
            # header exceeds the slot; never as ok
            assert s in (gpu.LGS_ST_CORRUPT, gpu.LGS_ST_NOSPACE), v.name


def test_decode_nospace(gpu):
    raw = corpus.fillseq(1).block(0)
    comp = gpu.encode(raw)
    res, st = gpu.decode_batch_host([comp, comp], [len(raw) - 1, len(raw)])
    assert list(st) == [gpu.LGS_ST_NOSPACE, gpu.LGS_ST_OK]
    assert res[1] == raw


def _device_roundtrip(c: corpus.Corpus):
    import torch
    from lcdb_amd import batch
    raw = batch.upload(c)
    comp = batch.encode_slots(raw)
    batch.encode(raw, comp)
    out = batch.decode_slots(c.len)
    st = torch.zeros(c.n, dtype=torch.uint8, device="cuda")
    batch.decode(comp, out, st)
    torch.cuda.synchronize()
    return raw, comp, out, st


def test_device_batch_c1_fillseq(gpu, digests):
    d = digests["C1_fillseq_1024x4KiB"]
    c = corpus.fillseq(1024)
    from lcdb_amd import batch
    raw, comp, out, st = _device_roundtrip(c)
    assert batch.digest(comp) == (d["comp_sha256"], d["comp_bytes"])
    assert bool((st == 1).all())
    assert batch.digest(out) == (d["raw_sha256"], d["raw_bytes"])


def test_device_batch_c3_mixed(gpu, digests):
    d = digests["C3_mixed"]
    c = corpus.mixed()
    from lcdb_amd import batch
    raw, comp, out, st = _device_roundtrip(c)
    assert batch.digest(comp) == (d["comp_sha256"], d["comp_bytes"])
    assert bool((st == 1).all())
    assert batch.digest(out) == (d["raw_sha256"], d["raw_bytes"])


def test_device_batch_c2_full_size(gpu, digests):
    # BASELINE config 2 at full size: 65 536 fillseq blocks; checksum of the
    # whole compressed corpus equals the reference's, round trip is exact.
    d = digests["C2_fillseq_65536x4KiB"]
    c = corpus.fillseq(65536)
    from lcdb_amd import batch
    raw, comp, out, st = _device_roundtrip(c)
    assert batch.digest(comp) == (d["comp_sha256"], d["comp_bytes"])
    assert int(st.sum().item()) == c.n
    assert batch.digest(out) == (d["raw_sha256"], d["raw_bytes"])


def test_device_batch_unaligned_offsets(gpu):
    import torch
    from lcdb_amd import batch
    c0 = corpus.concat(corpus.fillseq(37), corpus.random_blocks(11, 4096), corpus.fillseq(5, 16384))
    # re-pack with odd offsets: block i at 7*i + running total
    blocks = c0.blocks()
    off = np.zeros(len(blocks), dtype=np.uint64)
    at = 3
    for i, b in enumerate(blocks):
        off[i] = at
        at += len(b) + (i % 13)
    buf = np.zeros(at + 32, dtype=np.uint8)
    for i, b in enumerate(blocks):
        buf[int(off[i]):int(off[i]) + len(b)] = np.frombuffer(b, dtype=np.uint8)
    c = corpus.Corpus(buf, off, c0.len.copy())
    raw = batch.upload(c)
    comp = batch.encode_slots(raw)
    comp.off += torch.arange(c.n, device="cuda", dtype=torch.int64) % 7   # odd out slots
    comp.buf = torch.empty(comp.buf.numel() + 16, dtype=torch.uint8, device="cuda")
    batch.encode(raw, comp)
    torch.cuda.synchronize()
    ref = oracle.best()
    hc = batch.to_host(comp)
    for i in range(c.n):
        assert hc.block(i) == ref.encode(blocks[i]), i
    out = batch.decode_slots(c.len + 16)   # room for the odd shifts below
    out.off += (torch.arange(c.n, device="cuda", dtype=torch.int64) * 5) % 16
    out.buf = torch.empty(out.buf.numel() + 16, dtype=torch.uint8, device="cuda")
    st = torch.zeros(c.n, dtype=torch.uint8, device="cuda")
    batch.decode(comp, out, st)
    torch.cuda.synchronize()
    ho = batch.to_host(out)
    assert bool((st == 1).all())
    for i in range(c.n):
        assert ho.block(i) == blocks[i], i


def test_dropin_concurrent_threads(gpu):
    c = corpus.fillseq(64)
    ref = oracle.best()
    want = [ref.encode(b) for b in c.blocks()]
    errors = []

    def work(k):
        try:
            for i in range(k, c.n, 4):
                e = gpu.encode(c.block(i))
                if e != want[i] or gpu.decode(e) != c.block(i):
                    errors.append(i)
        except Exception as exc:   # pragma: no cover - reported below
            errors.append(repr(exc))

    ts = [threading.Thread(target=work, args=(k,)) for k in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors[:5]


def test_random_inputs_vs_oracle(gpu):
    import random
    rng = random.Random(7)
    ref = oracle.best()
    blocks = []
    for _ in range(300):
        n = rng.choice([rng.randrange(0, 40), rng.randrange(40, 4096), rng.randrange(4096, 65537)])
        kind = rng.randrange(3)
        if kind == 0:
            b = bytes(rng.randrange(256) for _ in range(n))
        elif kind == 1:
            alpha = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 5)))
            b = bytes(rng.choice(alpha) for _ in range(n))
        else:
            unit = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 30)))
            b = (unit * (n // max(1, len(unit)) + 1))[:n]
        blocks.append(b)
    outs = gpu.encode_batch_host(blocks)
    for b, o in zip(blocks, outs):
        assert o == ref.encode(b)


@pytest.mark.parametrize("kernel", _with_probe(["wave", "ring"], ["quad", "ops", "group", "chain"]))
def test_decode_kernel_variants_golden(gpu, vectors, kernel, force):
    # Every decode kernel (forced through lgs_set_option) against the
    # reference's accept/reject bit and output, on every golden stream.
    force("decoder", kernel)
    enc = [v for v in vectors if v.kind == 0]
    res, st = gpu.decode_batch_host([v.b for v in enc], [len(v.a) for v in enc])
    for v, o, s in zip(enc, res, st):
        assert s == gpu.LGS_ST_OK and o == v.a, (kernel, v.name)
    dec = [v for v in vectors if v.kind == 1]
    caps = [len(v.b) if v.ok else 1 << 17 for v in dec]
    res, st = gpu.decode_batch_host([v.a for v in dec], caps)
    for v, o, s in zip(dec, res, st):
        if v.ok:
            assert s == gpu.LGS_ST_OK and o == v.b, (kernel, v.name)
        else:
            assert s in (gpu.LGS_ST_CORRUPT, gpu.LGS_ST_NOSPACE), (kernel, v.name)


@pytest.mark.parametrize("kernels", _with_probe([("ring", "wave")], [("quad", "ops", "group", "chain")]))
def test_decode_kernels_c2_full_size(gpu, digests, force, kernels):
    import torch
    from lcdb_amd import batch
    d = digests["C2_fillseq_65536x4KiB"]
    c = corpus.fillseq(65536)
    raw = batch.upload(c)
    comp = batch.encode_slots(raw)
    batch.encode(raw, comp)
    for kernel in kernels:
        force("decoder", kernel)
        out = batch.decode_slots(c.len)
        st = torch.zeros(c.n, dtype=torch.uint8, device="cuda")
        batch.decode(comp, out, st)
        torch.cuda.synchronize()
        assert int(st.sum().item()) == c.n, kernel
        assert batch.digest(out) == (d["raw_sha256"], d["raw_bytes"]), kernel


def test_encode_small_batch_and_c1(gpu, vectors, digests):
    # All golden inputs of <= 4 608 B in one batch, then the full C1 corpus
    # on the device, against the reference's bytes.
    kernel = "wave"
    small = [v for v in vectors if v.kind == 0 and len(v.a) <= 4608]
    outs = gpu.encode_batch_host([v.a for v in small])
    for v, o in zip(small, outs):
        assert o == v.b, (kernel, v.name)
    # odd counts and single blocks (a wave's second half idle)
    for k in (1, 3):
        assert gpu.encode_batch_host([v.a for v in small[:k]]) == [v.b for v in small[:k]]
    import torch
    from lcdb_amd import batch
    d = digests["C1_fillseq_1024x4KiB"]
    c = corpus.fillseq(1024)
    raw = batch.upload(c)
    comp = batch.encode_slots(raw)
    batch.encode(raw, comp)
    torch.cuda.synchronize()
    assert batch.digest(comp) == (d["comp_sha256"], d["comp_bytes"]), kernel


@pytest.mark.parametrize("shift", [1, 2, 3, 7, 13])
def test_misaligned_blocks_c1_round_trip(gpu, digests, force, shift):
    # Every block (input, compressed stream and output) `shift` bytes off its
    # 16-byte alignment: the encoder's linear staging (16-byte loads at any
    # address) and every decoder's handling of odd stream and output offsets
    # against the pinned C1 digests; the ring decoder forced (C1 is below its
    # batch threshold), then the default wave decoder.
    import torch
    from lcdb_amd import batch
    d = digests["C1_fillseq_1024x4KiB"]
    c = corpus.fillseq(1024)
    buf = np.zeros(len(c.buf) + shift, dtype=np.uint8)
    buf[shift:] = c.buf
    cs = corpus.Corpus(buf, c.off + np.uint64(shift), c.len)
    raw = batch.upload(cs)
    comp = batch.encode_slots(raw)
    comp.off += shift
    batch.encode(raw, comp)
    hc = batch.to_host(comp)
    assert corpus.digest_of_digests(corpus.block_digests(hc.buf, hc.off, hc.len)) == d["comp_dd"]
    for kernel in ("ring", "auto"):
        force("decoder", kernel)
        out = batch.decode_slots(c.len + 16)
        out.off += shift
        st = torch.zeros(c.n, dtype=torch.uint8, device="cuda")
        batch.decode(comp, out, st)
        torch.cuda.synchronize()
        assert bool((st == 1).all()), kernel
        ho = batch.to_host(out)
        assert corpus.digest_of_digests(corpus.block_digests(ho.buf, ho.off, ho.len)) == d["raw_dd"]


def _guarded_page(hip, size):
    """A device mapping of `size` bytes (a multiple of the VMM granularity)
    followed by a reserved, unmapped granule: any read past the mapping
    faults.  Returns (base, release)."""
    import ctypes as C

    class Loc(C.Structure):
        _fields_ = [("type", C.c_int), ("id", C.c_int)]

    class Flags(C.Structure):
        _fields_ = [("compressionType", C.c_ubyte), ("gpuDirectRDMACapable", C.c_ubyte),
                    ("usage", C.c_ushort)]

    class Prop(C.Structure):
        _fields_ = [("type", C.c_int), ("requestedHandleType", C.c_int), ("location", Loc),
                    ("win32HandleMetaData", C.c_void_p), ("allocFlags", Flags)]

    class Access(C.Structure):
        _fields_ = [("location", Loc), ("flags", C.c_int)]

    dev = C.c_int()
    assert hip.hipGetDevice(C.byref(dev)) == 0
    prop = Prop(type=1, requestedHandleType=0, location=Loc(1, dev.value))   # pinned, device
    gran = C.c_size_t()
    assert hip.hipMemGetAllocationGranularity(C.byref(gran), C.byref(prop), 0) == 0
    g = gran.value
    size = (size + g - 1) // g * g
    base = C.c_void_p()
    assert hip.hipMemAddressReserve(C.byref(base), C.c_size_t(size + g), C.c_size_t(0),
                                    C.c_void_p(0), C.c_ulonglong(0)) == 0
    handle = C.c_void_p()
    assert hip.hipMemCreate(C.byref(handle), C.c_size_t(size), C.byref(prop), C.c_ulonglong(0)) == 0
    assert hip.hipMemMap(base, C.c_size_t(size), C.c_size_t(0), handle, C.c_ulonglong(0)) == 0
    acc = Access(location=Loc(1, dev.value), flags=3)                    # read-write
    assert hip.hipMemSetAccess(base, C.c_size_t(size), C.byref(acc), C.c_size_t(1)) == 0

    def release():
        hip.hipMemUnmap(base, C.c_size_t(size))
        hip.hipMemRelease(handle)
        hip.hipMemAddressFree(base, C.c_size_t(size + g))

    return base.value, size, release


def test_encode_block_flush_with_allocation_end(gpu):
    # lgs_encode_batch_dev promises no read slack, so a block
    # whose last byte is the last byte of its device memory must be encoded
    # from inside it (the staging reads a ragged last granule as the 16 bytes
    # ending at the block's end, and a block under 16 bytes a byte per lane).
    # Every length residue mod 16, each block flush with the end of a VMM
    # mapping whose next granule is reserved and unmapped (an overread faults
    # instead of reading a neighbour), against the reference encoder.
    import ctypes as C
    import torch
    from lcdb_amd import _native
    hip = C.CDLL("libamdhip64.so")
    ref = oracle.best()
    lib = _native.lib()
    rng = np.random.default_rng(0xF1)
    fill = corpus.fillseq(20)
    lengths = list(range(1, 49)) + [4096 + k for k in range(-16, 17)] + \
        [16384 + 9, 65536 - 5, 65536, 65536 + 7, 70001]
    base, size, release = _guarded_page(hip, 70001 + 16)
    try:
        # (The granule after the mapping is reserved and never mapped, by
        # construction; hipPointerGetAttributes reports reserved-unmapped
        # addresses as valid, so it cannot witness that.)
        for L in lengths:
            raw = bytes(fill.buf[:L]) if L <= len(fill.buf) else \
                bytes(rng.integers(0, 4, L, dtype=np.uint8))
            src = np.frombuffer(raw, dtype=np.uint8)
            assert hip.hipMemcpy(C.c_void_p(base + size - L), C.c_void_p(src.ctypes.data),
                                 C.c_size_t(L), 1) == 0
            off = torch.tensor([size - L], dtype=torch.int64, device="cuda")
            ln = torch.tensor([L], dtype=torch.int32, device="cuda")
            out = torch.zeros(gpu.encode_bound(L) + 16, dtype=torch.uint8, device="cuda")
            ooff = torch.zeros(1, dtype=torch.int64, device="cuda")
            olen = torch.zeros(1, dtype=torch.int32, device="cuda")
            s = torch.cuda.current_stream()
            _native.check(lib.lgs_encode_batch_dev(C.c_void_p(base), off.data_ptr(), ln.data_ptr(),
                                                   out.data_ptr(), ooff.data_ptr(),
                                                   olen.data_ptr(), 1, L, s.cuda_stream),
                          "lgs_encode_batch_dev")
            s.synchronize()
            got = out[:int(olen.item())].cpu().numpy().tobytes()
            assert got == ref.encode(raw), L
    finally:
        torch.cuda.synchronize()
        release()


def test_encode_c2_and_random(gpu, digests):
    # The encoder on the full C2 corpus, then on random, zero, periodic and
    # short inputs of every length class in one batch.
    import random
    import torch
    from lcdb_amd import batch
    d = digests["C2_fillseq_65536x4KiB"]
    c = corpus.fillseq(65536)
    raw = batch.upload(c)
    comp = batch.encode_slots(raw)
    batch.encode(raw, comp)
    torch.cuda.synchronize()
    assert batch.digest(comp) == (d["comp_sha256"], d["comp_bytes"])
    rng = random.Random(3)
    blocks = []
    for k in range(2001):
        n = rng.choice([rng.randrange(0, 20), rng.randrange(20, 600), rng.randrange(600, 4609)])
        kind = k % 4
        if kind == 0:
            b = bytes(rng.randrange(256) for _ in range(n))
        elif kind == 1:
            b = bytes(n)
        elif kind == 2:
            unit = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 70)))
            b = (unit * (n // len(unit) + 1))[:n]
        else:
            alpha = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 4)))
            b = bytes(rng.choice(alpha) for _ in range(n))
        blocks.append(b)
    outs = gpu.encode_batch_host(blocks)
    ref = oracle.best()
    for b, o in zip(blocks, outs):
        assert o == ref.encode(b)


@pytest.mark.parametrize("kernel", _with_probe(["ring"], ["quad", "ops", "group"]))
def test_decode_ring_c3_mixed_and_odd_slots(gpu, digests, force, kernel):
    # The LDS-ring decoder on C3 (4/16/64 KiB classes, half random: long
    # literals streamed through the input window, far copies) and on output
    # slots at odd offsets (flushes that are not line aligned, byte-exact
    # block ends next to the neighbouring block).
    import torch
    from lcdb_amd import batch
    force("decoder", kernel)
    d = digests["C3_mixed"]
    c = corpus.mixed()
    raw = batch.upload(c)
    comp = batch.encode_slots(raw)
    batch.encode(raw, comp)
    out = batch.decode_slots(c.len)
    st = torch.zeros(c.n, dtype=torch.uint8, device="cuda")
    batch.decode(comp, out, st)
    torch.cuda.synchronize()
    assert bool((st == 1).all())
    assert batch.digest(out) == (d["raw_sha256"], d["raw_bytes"])
    # odd slots, packed back to back (no slack between blocks)
    lens = c.len.astype(np.int64)
    off = np.zeros(c.n, dtype=np.int64)
    off[1:] = np.cumsum(lens[:-1])
    off += 3
    out2 = batch.Slots(torch.zeros(int(lens.sum()) + 3 + 16, dtype=torch.uint8, device="cuda"),
                       torch.from_numpy(off).cuda(), torch.zeros(c.n, dtype=torch.int32, device="cuda"),
                       torch.from_numpy(lens.astype(np.int32)).cuda(), int(lens.max()))
    st.zero_()
    batch.decode(comp, out2, st)
    torch.cuda.synchronize()
    assert bool((st == 1).all())
    host = out2.buf.cpu().numpy()
    ref = np.concatenate([np.frombuffer(c.block(k), dtype=np.uint8) for k in range(c.n)])
    assert np.array_equal(host[3:3 + len(ref)], ref)


def _varint(n: int) -> bytes:
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def _runahead_stream(want: int, copy_frac: float) -> bytes:
    # Output running ahead of input: 64-byte COPY2s (3 stream bytes each)
    # first, then 1-byte literals (2 stream bytes each).  The wave decoder
    # stages the stream at the top of its in-place LDS buffer; this shape
    # breaks the in-place bound when the copies are many, and must then be
    # decoded again from global memory, with the reference's result.
    ncopy = int((want - 4) * copy_frac) // 64
    nlit = want - 4 - 64 * ncopy
    s = bytearray(_varint(want))
    s += bytes([3 << 2]) + b"abcd"
    s += bytes([(63 << 2) | 2, 4, 0]) * ncopy
    for k in range(nlit):
        s += bytes([0, 0x41 + k % 26])
    return bytes(s)


def _header(s: bytes):
    # varint32 of coding.h:169-204 as snappy_decode_size reads it (None: bad)
    v = 0
    for k in range(min(5, len(s))):
        v |= (s[k] & 0x7F) << (7 * k)
        if not s[k] & 0x80:
            return v if v <= 0x7FFFFFFF else None
    return None


def _decode_ops_rejects_overflow_and_jumps(gpu, vectors, force):
    # The two-pass decoder (ops) on its own class, every outcome against the
    # reference: the golden compressed streams (corrupt ones included) at a
    # 4 608-byte capacity; 3 000 corruptions of fillseq blocks (byte flips,
    # truncations, appended bytes); streams with more ops than pass 1 records
    # (decoded by pass 2 from the stream alone); long literals that jump the
    # pass-1 ring past whole segments; the empty block.
    import random
    force("decoder", "ops")
    ref = oracle.best()
    rng = random.Random(11)
    cap = 4608
    streams = [v.a for v in vectors if v.kind == 1]
    good = [ref.encode(b) for b in corpus.fillseq(1000).blocks()]
    streams += good
    for _ in range(3000):
        s = bytearray(rng.choice(good))
        r = rng.randrange(4)
        if r == 0:
            for _ in range(rng.randrange(1, 4)):
                s[rng.randrange(len(s))] = rng.randrange(256)
        elif r == 1:
            del s[rng.randrange(1, len(s)):]
        elif r == 2:
            s += bytes(rng.randrange(256) for _ in range(rng.randrange(1, 6)))
        else:
            s[rng.randrange(min(len(s), 6))] ^= 1 << rng.randrange(8)
        streams.append(bytes(s))
    # > 1024 ops: 1-byte literals and 4-byte COPY1s (dist 1) alternating
    many = bytearray(_varint(4600))
    for _ in range(920):
        many += bytes([0, 0x61]) + bytes([(0 << 2) | 1, 1])
    streams += [bytes(many), bytes(many[:-1]), bytes(many[:-3]) + b"\x01\x09"]
    for _ in range(40):
        parts = []
        while sum(map(len, parts)) < 4000:
            k = rng.randrange(3)
            n = rng.randrange(1, 700)
            parts.append(bytes(rng.randrange(256) for _ in range(n)) if k == 0 else
                         bytes(n) if k == 1 else (b"key%05d" % rng.randrange(99999)) * (n // 8 + 1))
        raw = b"".join(parts)[:rng.randrange(3000, 4601)]
        streams.append(ref.encode(raw))
    streams += [b"\x00", b"", b"\x80", b"\x05\x10abcd"]
    res, st = gpu.decode_batch_host(streams, [cap] * len(streams))
    for k, (s, o, code) in enumerate(zip(streams, res, st)):
        exp = ref.decode(s) if s else None
        h = _header(s)
        if exp is not None and len(exp) <= cap:
            assert code == gpu.LGS_ST_OK and o == exp, k
        elif h is not None and h > cap:
            assert code == gpu.LGS_ST_NOSPACE, k
        else:
            assert code == gpu.LGS_ST_CORRUPT, k


if PROBE:   # the two-pass decoder exists in the probe library only
    test_decode_ops_rejects_overflow_and_jumps = pytest.mark.probe(
        _decode_ops_rejects_overflow_and_jumps)



@pytest.mark.parametrize("kernel", _with_probe([None, "ring"], ["quad", "ops", "group", "chain"]))
def test_decode_in_place_runahead(gpu, kernel, force):
    # One batch per output size, so each LDS class of the wave decoder (4, 16
    # and 64 KiB, chosen by the largest capacity) is the one that runs.
    if kernel:
        force("decoder", kernel)
    ref = oracle.best()
    for want in (4000, 4600, 16000, 16800, 60000, 66000):
        streams = []
        for frac in (0.1, 0.5, 0.9, 0.97):
            s = _runahead_stream(want, frac)
            streams += [s, s[:-1], s[:-2] + bytes([0xFC])]   # ok, truncated, bad tail
        res, st = gpu.decode_batch_host(streams, [want] * len(streams))
        for k, (s, o, code) in enumerate(zip(streams, res, st)):
            exp = ref.decode(s)
            if exp is None:
                assert code == gpu.LGS_ST_CORRUPT, (want, k)
            else:
                assert code == gpu.LGS_ST_OK and o == exp, (want, k)


def test_split_launch_all_classes(gpu, force):
    # A batch mixing every size class, large enough (>= 36 864 blocks) that
    # the 4 KiB class goes to the ring decoder: the launch is sorted into
    # classes on the device, each class in its own kernel.  Compressed bytes
    # equal the reference's (oracle, per block) and the unsplit launch's;
    # the round trip is exact, every status ok.
    import torch
    from lcdb_amd import batch
    ref = oracle.best()
    c = corpus.concat(corpus.fillseq(36600), corpus.random_blocks(400, 4096),
                      corpus.fillseq(40, block_size=16384), corpus.random_blocks(30, 16384),
                      corpus.fillseq(12, block_size=65536), corpus.random_blocks(6, 65536),
                      corpus.fillseq(3, block_size=100000), corpus.random_blocks(2, 70000))
    raw = batch.upload(c)
    comp = batch.encode_slots(raw)
    batch.encode(raw, comp)
    out = batch.decode_slots(c.len)
    st = torch.zeros(c.n, dtype=torch.uint8, device="cuda")
    batch.decode(comp, out, st)
    torch.cuda.synchronize()
    assert bool((st == 1).all())
    assert batch.digest(out) == batch.digest(raw)
    host = batch.to_host(comp)
    for k in list(range(0, c.n, 97)) + list(range(c.n - 100, c.n)):
        assert host.block(k) == ref.encode(c.block(k)), k
    force("split", "0")
    comp2 = batch.encode_slots(raw)
    batch.encode(raw, comp2)
    torch.cuda.synchronize()
    assert batch.digest(comp2) == batch.digest(comp)


def test_hbm_copy_probe_exact_and_rejects_misaligned(gpu):
    # The bench's yardstick copy: full tiles, a ragged tail, and the
    # alignment contract of lgs_hbm_copy_dev.
    import torch
    from lcdb_amd import _native
    lib = _native.lib()
    g = torch.Generator(device="cpu").manual_seed(7)
    for nbytes in (16, 16 * 1023, (16 << 10) * 5 + 48, 3 << 20):
        src = torch.randint(0, 256, (nbytes + 32,), dtype=torch.uint8, generator=g).cuda()
        dst = torch.zeros_like(src)
        assert lib.lgs_hbm_copy_dev(dst.data_ptr(), src.data_ptr(), nbytes, None) == 0
        torch.cuda.synchronize()
        assert torch.equal(dst[:nbytes], src[:nbytes]), nbytes
        assert int(dst[nbytes:].count_nonzero()) == 0, nbytes   # nothing past the end
    assert lib.lgs_hbm_copy_dev(dst.data_ptr(), src.data_ptr(), 24, None) != 0


def _lit(b: bytes) -> bytes:
    # literal tag, snappy.c:53-73 header forms (1-3 length bytes here)
    n = len(b) - 1
    if n < 60:
        return bytes([n << 2]) + b
    if n < 256:
        return bytes([60 << 2, n]) + b
    if n < 65536:
        return bytes([61 << 2, n & 255, n >> 8]) + b
    return bytes([62 << 2, n & 255, (n >> 8) & 255, n >> 16]) + b


def _copy2(length: int, dist: int) -> bytes:
    return bytes([((length - 1) << 2) | 2, dist & 255, dist >> 8])


@pytest.mark.parametrize("wide", _with_probe(["walk"], ["trips"]))
def test_decode_wide_far_copies_long_literals_and_rejects(gpu, force, wide):
    # Outputs over the 16 KiB class go to the wide decoders (a 32 KiB output
    # ring flushed to HBM, a 4 KiB stream ring refilled 2 KiB at a time; the
    # trip decoder moves up to 8 tags a step, the walk one).
    force("wide", wide)
    # Hand-made streams put copies beyond the ring (dist > 32 704, read back
    # from HBM), literals across many refills and flushes, and every kind of
    # reject at different depths; real 64 KiB / 100 KB / 300 KB blocks and
    # their corruptions follow.  Each against the reference's accept/reject
    # bit and bytes.
    import random
    rng = random.Random(11)
    ref = oracle.best()
    rnd = lambda n: bytes(rng.randrange(256) for _ in range(n))  # noqa: E731
    body = (_lit(rnd(40000)) + _copy2(64, 40000) + _copy2(64, 33000) + _copy2(20, 32705)
            + _lit(rnd(100)) + _copy2(60, 40200) + bytes([1 | (6 << 2) | (3 << 5), 0x10])
            + _lit(rnd(70000)) + _copy2(64, 65535) + _copy2(7, 3) + _copy2(64, 1))
    made = 40000 + 64 + 64 + 20 + 100 + 60 + 10 + 70000 + 64 + 7 + 64
    good = _varint(made) + body
    streams = [good,
               good[:-1],                                    # truncated tag
               good[:len(good) // 2],                        # truncated literal
               _varint(made + 1) + body,                     # stream ends short of want
               _varint(made - 1) + body,                     # op past want (snappy.c:323)
               _varint(40100) + _lit(rnd(40000)) + _copy2(64, 40001),   # dist > produced
               _varint(40100) + _lit(rnd(40000)) + bytes([2, 0, 0]),    # dist == 0
               _varint(70000) + _lit(rnd(70000))[:-5],       # literal past the stream
               _varint(5) + bytes([63 << 2, 1, 0, 0, 0]) + b"abcde"]     # 4-byte length
    for bs, n in ((65536, 3), (100000, 2), (300000, 1)):
        c = corpus.fillseq(n, block_size=bs, key0=bs)
        r = corpus.random_blocks(n, bs, seed=bs)
        for blk in [c.block(k) for k in range(c.n)] + [r.block(k) for k in range(r.n)]:
            s = ref.encode(blk)
            streams += [s, s[:-3]]
            for _ in range(4):
                k = rng.randrange(1, len(s))
                streams.append(s[:k] + bytes([rng.randrange(256)]) + s[k + 1:])
    # Through the drop-in too: outputs of 16 897 - 66 048 bytes
    # decode in the slot's mapped, coherent pinned memory, so far copies
    # there read flushed output back across PCIe.
    small = (_lit(rnd(40000)) + _copy2(64, 40000) + _copy2(64, 33000) + _copy2(20, 32705)
             + _lit(rnd(100)) + _copy2(60, 40200) + bytes([1 | (6 << 2) | (3 << 5), 0x10])
             + _lit(rnd(20000)) + _copy2(64, 60000) + _copy2(7, 3) + _copy2(64, 1))
    smade = 40000 + 64 + 64 + 20 + 100 + 60 + 10 + 20000 + 64 + 7 + 64
    assert 16896 < smade <= 66048
    sgood = _varint(smade) + small
    dropin = [sgood, sgood[:-1], sgood[:len(sgood) // 2], _varint(smade + 1) + small,
              _varint(smade - 1) + small, _varint(40100) + _lit(rnd(40000)) + _copy2(64, 40001)]
    for bs, n in ((65536, 2),):
        for blk in list(corpus.fillseq(n, block_size=bs, key0=7).blocks()) + list(
                corpus.random_blocks(n, bs, seed=5).blocks()):
            s = ref.encode(blk)
            dropin += [s, s[:-3]]
            for _ in range(3):
                k = rng.randrange(1, len(s))
                dropin.append(s[:k] + bytes([rng.randrange(256)]) + s[k + 1:])
    dok = 0
    for k, s in enumerate(dropin):
        exp = ref.decode(s)
        assert gpu.decode(s) == exp, k
        dok += exp is not None
    assert dok >= 5
    caps = [1 << 19] * len(streams)
    res, st = gpu.decode_batch_host(streams, caps)
    oks = 0
    for k, (s, o, code) in enumerate(zip(streams, res, st)):
        exp = ref.decode(s)
        if exp is None:
            assert code == gpu.LGS_ST_CORRUPT, k
        else:
            assert code == gpu.LGS_ST_OK and o == exp, k
            oks += 1
    assert oks >= 13


def _trip_stress_stream(rng, want: int) -> bytes:
    """Short literals and COPY1/COPY2s with small distances: many copies whose
    source is the output of the same trip (chains of dependent copies), some
    overlapping (dist < len) and some COPY4s, for the trip decoder's rounds."""
    out = bytearray()
    s = bytearray()
    while len(out) < want:
        r = rng.random()
        room = want - len(out)
        if len(out) < 8 or r < 0.35:
            n = min(rng.randrange(1, 61), room)
            b = bytes(rng.randrange(256) for _ in range(n))
            s += bytes([(n - 1) << 2]) + b
            out += b
            continue
        n = min(rng.randrange(4, 65), room)
        if n < 4:
            b = bytes(rng.randrange(256) for _ in range(n))
            s += bytes([(n - 1) << 2]) + b
            out += b
            continue
        if r < 0.45:
            d = rng.randrange(1, min(n, len(out)) + 1)          # overlapping
        else:
            d = rng.randrange(n, min(len(out), 400) + 1) if len(out) >= n else len(out)
        d = max(1, min(d, len(out)))
        if r > 0.97:
            s += bytes([((n - 1) << 2) | 3]) + d.to_bytes(4, "little")
        elif d < 2048 and 4 <= n <= 11 and r < 0.7:
            s += bytes([1 | ((n - 4) << 2) | ((d >> 8) << 5), d & 255])
        else:
            s += bytes([((n - 1) << 2) | 2, d & 255, d >> 8])
        for k in range(n):
            out.append(out[len(out) - d])
    return _varint(len(out)) + bytes(s), bytes(out)


@pytest.mark.parametrize("wide", _with_probe(["walk"], ["trips", "group"]))
def test_decode_wide_dependent_copies_and_c3(gpu, digests, force, wide):
    # The wide class (outputs over 16 KiB) on C3 (its 64 KiB fillseq and
    # random classes among the others) and on hand-made streams dense in
    # copies that read this trip's own output, against the reference.
    import random
    import torch
    from lcdb_amd import batch
    force("wide", wide)
    d = digests["C3_mixed"]
    c = corpus.mixed()
    raw = batch.upload(c)
    comp = batch.encode_slots(raw)
    batch.encode(raw, comp)
    out = batch.decode_slots(c.len)
    st = torch.zeros(c.n, dtype=torch.uint8, device="cuda")
    batch.decode(comp, out, st)
    torch.cuda.synchronize()
    assert bool((st == 1).all())
    assert batch.digest(out) == (d["raw_sha256"], d["raw_bytes"])
    rng = random.Random(2027)
    ref = oracle.best()
    streams, exps = [], []
    for want in (17000, 40000, 65536, 66000, 120000):
        for _ in range(3):
            s, o = _trip_stress_stream(rng, want)
            assert ref.decode(s) == o
            streams += [s, s[:-1]]
            exps += [o, ref.decode(s[:-1])]
            k = rng.randrange(len(s) // 2, len(s))
            bad = s[:k] + bytes([rng.randrange(256)]) + s[k + 1:]
            streams.append(bad)
            exps.append(ref.decode(bad))
    res, st = gpu.decode_batch_host(streams, [1 << 18] * len(streams))
    for k, (o, code, exp) in enumerate(zip(res, st, exps)):
        if exp is None:
            assert code == gpu.LGS_ST_CORRUPT, k
        else:
            assert code == gpu.LGS_ST_OK and o == exp, k


def _group_streams(rng, ref):
    """Streams for the chain decoder's 64-tag batches and the workgroup
    decoder's windows (4 096 stream bytes, 8 192 output bytes each): real
    4 / 16 / 64 KiB blocks, dependent-copy
    stress streams, long literals crossing windows, outputs that cut windows
    (64-byte copies of dist 1: 21 output bytes per stream byte), every reject
    placed in the first, a middle and the last window, and their corruptions."""
    streams = []
    for c in (corpus.fillseq(6), corpus.fillseq(3, 16384, key0=9), corpus.fillseq(3, 65536, key0=3),
              corpus.random_blocks(3, 4096), corpus.random_blocks(2, 65536, seed=9)):
        for b in c.blocks():
            s = ref.encode(b)
            streams += [s, s[:-1], s[:-5]]
            for _ in range(6):
                k = rng.randrange(len(s))
                streams.append(s[:k] + bytes([rng.randrange(256)]) + s[k + 1:])
    for want in (100, 4000, 9000, 16000, 40000, 66000):
        for _ in range(3):
            s, _o = _trip_stress_stream(rng, want)
            streams += [s, s[:-1]]
            k = rng.randrange(1, len(s))
            streams.append(s[:k] + bytes([rng.randrange(256)]) + s[k + 1:])
    rnd = lambda n: bytes(rng.randrange(256) for _ in range(n))  # noqa: E731
    # runs: one literal, then 64-byte copies of dist 1 (window output cut)
    for want in (9000, 30000, 66000):
        n = (want - 1) // 64
        body = _lit(b"z") + _copy2(64, 1) * n + _lit(b"q" * (want - 1 - 64 * n))
        streams += [_varint(want) + body, _varint(want + 1) + body, _varint(want - 1) + body]
    # long literals straddling windows, between copies
    for n in (4090, 4100, 8191, 8192, 8193, 20000, 65000):
        lit = rnd(n)
        body = _lit(lit[:10]) + _copy2(8, 10) + _lit(lit) + _copy2(64, n // 2 + 1) + _lit(b"end")
        want = 10 + 8 + n + 64 + 3
        if want <= 66048:
            streams += [_varint(want) + body, _varint(want) + body[:-2]]
    # rejects in the first / a middle / the last window
    base = _lit(rnd(3000)) + _copy2(60, 2900) * 40 + _lit(rnd(100))
    made = 3000 + 60 * 40 + 100
    for bad in (bytes([2, 0, 0]),                          # dist 0
                _copy2(64, 60000),                         # dist > made
                bytes([(63 << 2) | 3]) + (2**31).to_bytes(4, "little"),   # dist >= 2^31
                bytes([63 << 2]) + b"\xff\xff\xff\x7f",    # literal length 2^31
                bytes([62 << 2, 0xff, 0xff]),              # header past the stream
                _copy2(64, 1)):                            # past want
        for pre in (b"", base, base * 3):
            pm = made * (len(pre) // len(base)) if pre else 0
            streams.append(_varint(pm + 4) + pre + bad + _lit(b"tail"))
    streams += [b"", b"\x00", b"\x80", b"\x00\x00", b"\x01\x00a", b"\x05\x10abcd",
                _varint(3) + _lit(b"ab") + bytes([1, 1]), _varint(0) + _lit(b"x")]
    return streams


@pytest.mark.parametrize("kernel,cap", [("wave", 4608), ("wave", 16896), ("wave", 66048)] + (
    [pytest.param("group", c, marks=pytest.mark.probe) for c in (4608, 16896, 66048)] +
    [pytest.param("chain", c, marks=pytest.mark.probe) for c in (4608, 16896)] if PROBE
    else []))
def test_decode_small_batch_kernels_and_rejects(gpu, force, kernel, cap):
    # The wave decoder (and, in the probe library, the workgroup and chain
    # decoders) forced on every stream of _group_streams, at each LDS class,
    # against the reference's bytes and accept/reject bit (a header beyond
    # the capacity is LGS_ST_NOSPACE, as in every decoder).
    import random
    force("decoder", kernel)
    rng = random.Random(cap)
    ref = oracle.best()
    streams = _group_streams(rng, ref)
    res, st = gpu.decode_batch_host(streams, [cap] * len(streams))
    oks = 0
    for k, (s, o, code) in enumerate(zip(streams, res, st)):
        exp = ref.decode(s) if s else None
        h = _header(s)
        if h is not None and h > cap:
            assert code == gpu.LGS_ST_NOSPACE, k
        elif exp is None:
            assert code == gpu.LGS_ST_CORRUPT, k
        else:
            assert code == gpu.LGS_ST_OK and o == exp, k
            oks += 1
    assert oks >= 20


def test_decode_dropin_small_batch_path(gpu):
    # Single blocks through the drop-in (the wave decoder; the 64 KiB class
    # the wide walk), from the slot's mapped pinned memory.
    import random
    rng = random.Random(5)
    ref = oracle.best()
    for s in _group_streams(rng, ref)[:400]:
        assert gpu.decode(s) == (ref.decode(s) if s else None)


def _op_stream(rng, want_max=4608, max_ops=None):
    """A valid Snappy stream built op by op (random literals and copies of
    every tag form, overlapping and chained copies), with its output."""
    out = bytearray()
    body = bytearray()
    nops = 0
    target = rng.randrange(1, want_max + 1)
    while len(out) < target and (max_ops is None or nops < max_ops):
        room = target - len(out)
        if not out or rng.random() < 0.35:
            n = min(room, rng.choice([1, 2, 3, rng.randrange(1, 17), rng.randrange(1, 70),
                                      rng.randrange(1, 300)]))
            lit = bytes(rng.randrange(256) for _ in range(n))
            m = n - 1
            if m < 60:
                body.append(m << 2)
            else:
                nb = 1 if m < 256 else 2
                body.append((59 + nb) << 2)
                body += m.to_bytes(nb, "little")
            body += lit
            out += lit
        else:
            n = min(room, rng.choice([rng.randrange(4, 12), rng.randrange(1, 65), 64]))
            d = rng.choice([1, 2, 3, rng.randrange(1, 9), rng.randrange(1, len(out) + 1)])
            d = min(d, len(out))
            form = rng.random()
            if 4 <= n <= 11 and d < 2048 and form < 0.4:
                body += bytes([((d >> 8) << 5) | ((n - 4) << 2) | 1, d & 0xFF])
            elif form < 0.9:
                body += bytes([((n - 1) << 2) | 2]) + d.to_bytes(2, "little")
            else:
                body += bytes([((n - 1) << 2) | 3]) + d.to_bytes(4, "little")
            for _ in range(n):
                out.append(out[-d])
        nops += 1
    return _varint(len(out)) + bytes(body), bytes(out)


@pytest.mark.parametrize("kernel", _with_probe(["auto", "wave"], ["ops"]))
def test_op_streams(gpu, force, kernel):
    # Streams built op by op: every tag form, overlapping copies (dist < len),
    # chains of copies of copies, streams of many tiny ops, and their
    # truncations and corruptions -- against the reference's decode.  "auto"
    # repeats them past the ring decoder's threshold (36 864 blocks); "wave"
    # forces the wave decoder; the probe library's two-pass decoder ("ops",
    # DESIGN 4.2) takes the same streams, including more ops than its first
    # pass records (its slow path).
    import random
    force("decoder", kernel)
    rng = random.Random(606)
    ref = oracle.best()
    streams, want = [], []
    for _ in range(600):
        s, o = _op_stream(rng)
        streams.append(s)
        want.append(len(o))
    for _ in range(20):                       # > 512 tags: the slow path
        body = bytearray()
        out = bytearray()
        for k in range(rng.randrange(513, 900)):
            if k % 2 == 0 or not out:
                b = rng.randrange(256)
                body += bytes([0, b])
                out.append(b)
            else:
                body += bytes([((1 - 1) << 2) | 2, 1, 0])
                out.append(out[-1])
        streams.append(_varint(len(out)) + bytes(body))
        want.append(len(out))
    bad = []
    for s in streams[:200]:
        b = bytearray(s)
        b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
        bad.append(bytes(b))
        bad.append(s[:-1])
    streams += bad
    want += [4608] * len(bad)
    reps = 37000 // len(streams) + 1 if kernel == "auto" else 1
    res, st = gpu.decode_batch_host(streams * reps, want * reps)
    for k, (s, o, code) in enumerate(zip(streams * reps, res, st)):
        exp = ref.decode(s)
        if exp is None or len(exp) > (want * reps)[k]:
            assert code in (gpu.LGS_ST_CORRUPT, gpu.LGS_ST_NOSPACE), k
            if exp is None:
                assert code == gpu.LGS_ST_CORRUPT, k
        else:
            assert code == gpu.LGS_ST_OK and o == exp, k

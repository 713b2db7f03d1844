"""GPU parity of the block-framing rows (§8(f) 1-3) through the C ABI:
CRC32C trailers, the batched data-block writer and the batched block reader,
against the oracle (oracle/table_oracle.c, itself pinned to the reference in
test_table_oracle.py) and against the reference's own .ldb files and
ldb_read_block results (oracle/harness)."""
from __future__ import annotations

import random
import struct

import numpy as np
import pytest

import oracle
import table_io
from table_io import LDB_OK

pytestmark = pytest.mark.gpu

RFC3720 = bytes([
    0x01, 0xc0, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
    0x00, 0x00, 0x00, 0x00, 0x14, 0x00, 0x00, 0x00, 0x00, 0x00, 0x04, 0x00,
    0x00, 0x00, 0x00, 0x14, 0x00, 0x00, 0x00, 0x18, 0x28, 0x00, 0x00, 0x00,
    0x00, 0x00, 0x00, 0x00, 0x02, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00])


@pytest.fixture(scope="module")
def tab(gpu):
    from lcdb_amd import table
    return table


def _device_pack(blocks, torch, shift: int = 0):
    """Blocks packed at 16-aligned offsets (+ shift), 16 bytes of slack."""
    offs, at = [], 0
    for b in blocks:
        at = (at + 15) // 16 * 16 + shift
        offs.append(at)
        at += len(b)
    buf = np.zeros(at + 64, dtype=np.uint8)
    for o, b in zip(offs, blocks):
        buf[o:o + len(b)] = np.frombuffer(b, dtype=np.uint8)
    t = torch.from_numpy(buf).cuda()
    off = torch.tensor(offs, dtype=torch.int64).cuda()
    ln = torch.tensor([len(b) for b in blocks], dtype=torch.int32).cuda()
    return t, off, ln


def _crc_cases():
    rng = random.Random(0x7ab1e)
    cases = [bytes(32), b"\xff" * 32, bytes(range(32)), bytes(range(31, -1, -1)), RFC3720,
             b"\xaa" * ((1 << 20) + 17), b"", b"a", b"ab", b"abc", b"abcd"]
    cases += [rng.randbytes(n) for n in list(range(0, 70)) + [4095, 4096, 4097, 8191, 8192,
                                                                 12289, 65536, 65541, 200003]]
    return cases


@pytest.mark.parametrize("shift", [0, 1, 3, 4, 6, 8, 13, 15])
@pytest.mark.parametrize("with_type", [False, True])
def test_crc32c_batch_vs_oracle(tab, shift, with_type):
    import torch
    cases = _crc_cases()
    buf, off, ln = _device_pack(cases, torch, shift)
    types = [i % 3 for i in range(len(cases))]
    d_type = torch.tensor(types, dtype=torch.uint8).cuda() if with_type else None
    for masked in (False, True):
        got = tab.crc32c_batch(buf, off, ln, d_type, masked).cpu().numpy().astype(np.uint32)
        for i, b in enumerate(cases):
            c = oracle.crc32c(b)
            if with_type:
                c = oracle.crc32c(bytes([types[i]]), c)
            if masked:
                c = oracle.crc32c_mask(c)
            assert int(got[i]) == c, (i, len(b), masked)
    # The reference's own known answers (t-crc32c.c:39-54, 108).
    if not with_type:
        got = tab.crc32c_batch(buf, off, ln, None, False).cpu().numpy().astype(np.uint32)
        assert [int(x) for x in got[:6]] == [0x8a9136aa, 0x62a8ab43, 0x46dd794e, 0x113fdb5c,
                                             0xd9963a56, 0xb0d7025a]


def test_crc32c_flush_with_allocation_end(tab):
    # Blocks whose last byte is the last byte of a device mapping followed by
    # an unmapped granule: the CRC reads only granules holding block bytes
    # (the type byte comes from its own array), so none of these faults.
    import ctypes as C
    import torch
    from test_gpu_parity import _guarded_page
    hip = C.CDLL("libamdhip64.so")
    rng = random.Random(0x9a4d)
    lengths = [1, 3, 4, 15, 16, 17, 63, 64, 65, 4095, 4096, 4097, 9000]
    base, size, release = _guarded_page(hip, 9000 + 64)
    try:
        for L in lengths:
            raw = rng.randbytes(L)
            src = np.frombuffer(raw, dtype=np.uint8)
            assert hip.hipMemcpy(C.c_void_p(base + size - L), C.c_void_p(src.ctypes.data),
                                 C.c_size_t(L), 1) == 0
            off = torch.tensor([size - L], dtype=torch.int64, device="cuda")
            ln = torch.tensor([L], dtype=torch.int32, device="cuda")
            ty = torch.tensor([1], dtype=torch.uint8, device="cuda")
            crc = torch.zeros(1, dtype=torch.int32, device="cuda")
            for d_type in (None, ty):
                s = torch.cuda.current_stream()
                tab.check(tab._L.lgs_crc32c_batch_dev(
                    C.c_void_p(base), off.data_ptr(), ln.data_ptr(),
                    d_type.data_ptr() if d_type is not None else None, 0, crc.data_ptr(), 1,
                    s.cuda_stream), "lgs_crc32c_batch_dev")
                s.synchronize()
                want = oracle.crc32c(raw)
                if d_type is not None:
                    want = oracle.crc32c(b"\x01", want)
                assert int(crc.item()) & 0xffffffff == want, (L, d_type is not None)
    finally:
        torch.cuda.synchronize()
        release()


@pytest.fixture(scope="module")
def ref_tables(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("gldb")
    out = {}
    for entries, bs in [(20000, 4096), (1500, 256), (12000, 65536)]:
        path = table_io.build_table(tmp, entries, bs)
        d = table_io.dump_blocks(path, str(tmp / f"dump_{bs}.bin"), verify=True)
        out[bs] = (path, open(path, "rb").read(), d)
    return out


@pytest.mark.parametrize("bs", [4096, 256, 65536])
def test_write_blocks_host_reproduces_reference_file(tab, ref_tables, bs):
    path, file, d = ref_tables[bs]
    ndata = d.n - 2
    region, hoff, hsize, end = tab.write_blocks_host(d.contents[:ndata], tab.LGS_SNAPPY_COMPRESSION)
    assert end == d.metaindex[0]
    assert region == file[:end]
    assert np.array_equal(hoff, d.off[:ndata]) and np.array_equal(hsize, d.size[:ndata])
    # The metaindex and index blocks too, each framed at its own offset.
    for k in (ndata, ndata + 1):
        r, ho, hs, e = tab.write_blocks_host([d.contents[k]], tab.LGS_SNAPPY_COMPRESSION,
                                             int(d.off[k]))
        assert int(ho[0]) == int(d.off[k]) and int(hs[0]) == int(d.size[k])
        assert r == file[int(d.off[k]):e]


def _mixed_blocks():
    rng = random.Random(0xb10c)
    from lcdb_amd import corpus
    c = corpus.fillseq(64)
    blocks = [c.block(i) for i in range(c.n)]
    blocks += [rng.randbytes(n) for n in (0, 1, 2, 3, 4, 17, 4096, 16384, 65536, 70000)]
    blocks += [bytes(n) for n in (0, 1, 5, 100, 65536, 131073)]
    half = rng.randbytes(2000)
    blocks += [half + bytes(len(half) // 6), half + bytes(len(half) // 7 + 40)]   # 12.5 % edge
    rng.shuffle(blocks)
    return blocks


@pytest.mark.parametrize("compression", [1, 0])
def test_write_blocks_vs_oracle(tab, compression):
    blocks = _mixed_blocks()
    want = oracle.table_write_blocks(blocks, compression, 12345)
    got = tab.write_blocks_host(blocks, compression, 12345)
    assert got[3] == want[3]
    assert got[0] == want[0]
    assert np.array_equal(got[1], want[1]) and np.array_equal(got[2], want[2])


def _small_blocks(n):
    """n blocks of at most 4608 bytes (the fused write's range): fillseq
    blocks, random and zero blocks of every awkward length, the 12.5 % edge."""
    rng = random.Random(0x5a11)
    from lcdb_amd import corpus
    c = corpus.fillseq(max(n // 2, 1))
    blocks = [c.block(i) for i in range(n // 2)]
    while len(blocks) < n:
        k = rng.randrange(6)
        if k == 0:
            blocks.append(rng.randbytes(rng.choice([0, 1, 2, 3, 4, 5, 16, 17, 63, 64, 65, 4608])))
        elif k == 1:
            blocks.append(bytes(rng.randrange(4609)))
        elif k == 2:
            half = rng.randbytes(rng.randrange(8, 3800))
            pad = len(half) // 6 + rng.randrange(-3, 4)
            blocks.append(half + bytes(max(pad, 0)))
        else:
            blocks.append(c.block(rng.randrange(c.n))[:rng.randrange(4609)])
    rng.shuffle(blocks)
    return blocks


@pytest.mark.parametrize("n", [1, 63, 65, 5000])
def test_write_small_blocks_vs_oracle(tab, n):
    # Blocks <= 4608 B (the one-stride encode slots), host and device entry.
    import torch
    blocks = _small_blocks(n)
    assert max(len(b) for b in blocks) <= 4608
    want = oracle.table_write_blocks(blocks, 1, 777)
    got = tab.write_blocks_host(blocks, 1, 777)
    assert got[3] == want[3]
    assert got[0] == want[0]
    assert np.array_equal(got[1], want[1]) and np.array_equal(got[2], want[2])
    buf, off, ln = _device_pack(blocks, torch, 3)
    d_file, hoff, hsize, end = tab.write_blocks(buf, off, ln, 1, 777)
    torch.cuda.synchronize()
    assert int(end.cpu()[0]) == want[3]
    assert d_file[:want[3] - 777].cpu().numpy().tobytes() == want[0]
    assert np.array_equal(hoff.cpu().numpy().astype(np.uint64), want[1])
    assert np.array_equal(hsize.cpu().numpy().astype(np.uint64), want[2])


def test_write_blocks_device_fillseq(tab):
    import torch
    from lcdb_amd import corpus
    c = corpus.fillseq(1024)
    blocks = [c.block(i) for i in range(c.n)]
    buf, off, ln = _device_pack(blocks, torch, 5)
    d_file, hoff, hsize, end = tab.write_blocks(buf, off, ln, 1, 0)
    torch.cuda.synchronize()
    e = int(end.cpu()[0])
    want = oracle.table_write_blocks(blocks, 1, 0)
    assert e == want[3]
    assert d_file[:e].cpu().numpy().tobytes() == want[0]
    assert np.array_equal(hoff.cpu().numpy().astype(np.uint64), want[1])


def _read_all(tab, file, off, size, caps, verify):
    return tab.read_blocks_host(file, off, size, caps, verify)


@pytest.mark.parametrize("bs", [4096, 256, 65536])
@pytest.mark.parametrize("verify", [True, False])
def test_read_blocks_host_matches_reference(tab, ref_tables, bs, verify):
    path, file, d = ref_tables[bs]
    caps = [max(len(x), 1) for x in d.contents]
    res, st = tab.read_blocks_host(file, d.off, d.size, caps, verify)
    for i in range(d.n):
        assert table_io.same_outcome(int(st[i]), d.rc[i]), (i, st[i], d.rc[i])
        assert res[i] == d.contents[i], i


@pytest.mark.parametrize("overlap", ["1", "0"])
@pytest.mark.parametrize("verify", [True, False])
def test_read_blocks_corrupted_matches_reference(tab, ref_tables, tmp_path, verify, overlap, force):
    # overlap: the trailer CRCs in their own pass beside the decoder (the
    # default) or inside the type dispatch.
    force("verify_overlap", overlap)
    path, file, d = ref_tables[4096]
    for seed in range(3):
        bad = table_io.corrupt(file, 0, d.metaindex[0], 60, 100 + seed)
        p = tmp_path / f"bad{seed}.ldb"
        p.write_bytes(bad)
        handles = np.stack([d.off, d.size], axis=1)
        dd = table_io.dump_blocks(str(p), str(tmp_path / f"d{seed}.bin"), verify, handles)
        res, st = tab.read_blocks_host(bad, d.off, d.size, [1 << 17] * d.n, verify)
        for i in range(d.n):
            assert table_io.same_outcome(int(st[i]), dd.rc[i]), (seed, i, st[i], dd.rc[i])
            if dd.rc[i] == LDB_OK:
                assert res[i] == dd.contents[i]


@pytest.mark.parametrize("verify,overlap", [(True, "1"), (True, "0"), (False, "1")])
def test_read_blocks_bad_handles_and_types(tab, ref_tables, tmp_path, verify, overlap, force):
    # verify False: the checks one lane per handle (check_lane_kernel).
    force("verify_overlap", overlap)
    path, file, d = ref_tables[256]
    n = len(file)
    handles = [(0, n), (n - 4, 0), (n - 5, 0), (n, 0), (n + 10, 3),
               (int(d.off[1]), int(d.size[1]) + 1), (int(d.off[2]) + 1, int(d.size[2])), (1, 2),
               (0, 0), (2**64 - 100, 50), (5, 2**64 - 3)]
    dd = table_io.dump_blocks(path, str(tmp_path / "h.bin"), verify, handles)
    off = np.array([h[0] for h in handles], dtype=np.uint64)
    size = np.array([h[1] for h in handles], dtype=np.uint64)
    res, st = tab.read_blocks_host(file, off, size, [1 << 17] * len(handles), verify)
    for i in range(len(handles)):
        assert table_io.same_outcome(int(st[i]), dd.rc[i]), (i, st[i], dd.rc[i])
        assert res[i] == (dd.contents[i] if dd.rc[i] == LDB_OK else None)
    # Type byte 2 with a valid checksum: "bad block type" (format.c:263-267);
    # a snappy type over raw bytes: corrupt stream; too small a slot: NOSPACE.
    # A wrong trailer CRC wins over every later outcome (format.c:203-211):
    # raw, bad type, snappy, too small a slot.
    blocks = [b"x" * 300, b"\x05hello", b"y" * 5000, b"z" * 100, b"w" * 50, b"\x05hello",
              b"v" * 5000, bytes(range(40)), b"u" * 4096]
    types = [2, 1, 0, 0, 2, 1, 0, 0, 0]
    wrong = [0, 0, 0, 1, 1, 1, 1, 0, 0]
    region = bytearray()
    offs = []
    for b, ty, bad in zip(blocks, types, wrong):
        offs.append(len(region))
        c = oracle.crc32c_mask(oracle.crc32c(bytes([ty]), oracle.crc32c(b))) ^ bad
        region += b + bytes([ty]) + c.to_bytes(4, "little")
    sizes = np.array([len(b) for b in blocks], dtype=np.uint64)
    offs = np.array(offs, dtype=np.uint64)
    caps = [4096] * len(blocks)
    res, st = tab.read_blocks_host(bytes(region), offs, sizes, caps, verify)
    for i in range(len(blocks)):
        ost, ores = oracle.table_read_block(bytes(region), int(offs[i]), int(sizes[i]), verify, caps[i])
        assert int(st[i]) == ost and res[i] == ores, i
    first = [tab.LGS_ST_BADTYPE, tab.LGS_ST_CORRUPT, tab.LGS_ST_NOSPACE]
    assert list(st) == first + ([tab.LGS_ST_BADCRC] * 4 if verify else [tab.LGS_ST_OK] + first) + \
        [tab.LGS_ST_OK] * 2                       # raw blocks of 40 and 4 096 bytes


@pytest.mark.parametrize("bs", [4096, 256, 65536])
def test_table_index_then_batched_read(tab, ref_tables, bs):
    """ldb_table_open's view (footer -> index block -> data-block handles and
    separator keys) matches the reference's index walk; the batched read of
    those handles returns every data block as ldb_read_block does."""
    path, file, d = ref_tables[bs]
    ndata = d.n - 2
    for paranoid in (True, False):
        handles, keys, fh, st = tab.index_host(file, paranoid, internal_keys=True)
        assert st == tab.LGS_ST_OK and fh is None       # no filter policy in these tables
        assert handles == list(zip(d.off[:ndata].tolist(), d.size[:ndata].tolist()))
        assert keys == [k for k, _ in table_io.block_entries(d.contents[-1])]
    off = np.array([h[0] for h in handles], dtype=np.uint64)
    size = np.array([h[1] for h in handles], dtype=np.uint64)
    res, st = tab.read_blocks_host(file, off, size, [max(len(x), 1) for x in d.contents[:ndata]])
    assert all(int(x) == tab.LGS_ST_OK for x in st)
    assert res == d.contents[:ndata]


def test_table_index_filter_handle(tab, tmp_path):
    path = table_io.build_table(tmp_path, 6000, 4096, bloom_bits=10)
    file = open(path, "rb").read()
    d = table_io.dump_blocks(path, str(tmp_path / "d.bin"), True)
    handles, keys, fh, st = tab.index_host(file, True, internal_keys=True)
    assert st == tab.LGS_ST_OK and len(handles) == d.n - 2
    assert fh == table_io.filter_handle(d.contents[-2])
    assert tab.index_host(file, True, filter_name="filter.other")[2] is None


def test_table_index_damaged_files(tab, ref_tables):
    path, file, d = ref_tables[256]
    ndata = d.n - 2
    corrupt = tab.LGS_ST_CORRUPT
    assert tab.index_host(file[:47])[3] == corrupt                      # table.c:127-128
    assert tab.index_host(b"")[3] == corrupt
    assert tab.index_host(file[:-1] + bytes([file[-1] ^ 1]))[3] == corrupt   # magic
    # An index handle past the end: the read's I/O status (format.c:195-198).
    io_, is_ = d.index
    bad = bytearray(file)
    footer = bytearray(file[-48:])
    mo, ms = d.metaindex
    def v(x):
        out = bytearray()
        while x >= 128:
            out.append((x & 127) | 128)
            x >>= 7
        out.append(x)
        return out
    enc = v(mo) + v(ms) + v(len(file) + 100) + v(is_)
    footer[:len(enc)] = enc
    bad[-48:] = footer
    assert tab.index_host(bytes(bad))[3] == tab.LGS_ST_IOERR
    # A flipped byte inside the index block: its checksum, when verified.
    flip = bytearray(file)
    flip[io_ + 3] ^= 0x40
    handles, _, _, st = tab.index_host(bytes(flip), paranoid_checks=True)
    assert st == tab.LGS_ST_BADCRC and handles == []
    # A cap too small is an error, not a truncated answer.
    with pytest.raises(Exception):
        tab.index_host(file, cap=ndata - 1)


def test_table_index_corrupt_entries_vs_reference(tab, ref_tables, tmp_path):
    """Index blocks with damaged entries (stored raw with a valid checksum, so
    the block reads): the walk stops where lcdb's own block iterator stops
    (block.c:80-126, 255-297), with the same handles before it."""
    path, file, d = ref_tables[256]
    contents = d.contents[-1]
    io_ = d.index[0]
    offs = table_io.entry_offsets(contents)
    nr = struct.unpack_from("<I", contents, len(contents) - 4)[0]
    cases = {}
    k = len(offs) // 2
    b = bytearray(contents)
    b[offs[k]] = 0x7f                                    # shared > the previous key's size
    cases["shared"] = bytes(b)
    b = bytearray(contents)
    b[offs[k] + 2] = 0x7f                                # value runs into the restart array
    cases["value_len"] = bytes(b)
    b = bytearray(contents)
    b[offs[-1] + 1] = 0xff                               # an unterminated varint at the end
    b[offs[-1] + 2] = 0xff
    cases["varint"] = bytes(b)
    b = bytearray(contents)
    struct.pack_into("<I", b, len(b) - 4, 0)             # no restarts: an empty block
    cases["no_restarts"] = bytes(b)
    b = bytearray(contents)
    struct.pack_into("<I", b, len(b) - 4, len(b))        # more restarts than fit
    cases["restarts"] = bytes(b)
    cases["intact_raw"] = contents
    for name, cont in cases.items():
        img = table_io.with_raw_index(file, io_, d.metaindex, cont)
        p = tmp_path / f"{name}.ldb"
        p.write_bytes(img)
        ref = table_io.dump_blocks(str(p), str(tmp_path / f"{name}.bin"), True)
        want = list(zip(ref.off[:ref.n - 2].tolist(), ref.size[:ref.n - 2].tolist()))
        handles, keys, _, st = tab.index_host(img, True, internal_keys=False)
        assert handles == want, name
        ok = name in ("no_restarts", "intact_raw")
        assert st == (tab.LGS_ST_OK if ok else tab.LGS_ST_CORRUPT), (name, st)
    assert nr > 1


def test_host_paths_chunked_c2_scale(tab):
    """The host-buffer table paths at BASELINE scale, where they run as a
    two-stream chunk pipeline: the region equals the device path's byte for
    byte, and reading it back through the host path returns every block."""
    import torch
    from lcdb_amd import batch, corpus
    c = corpus.fillseq(65536)
    blocks = c.blocks()
    region, hoff, hsize, end = tab.write_blocks_host(blocks, tab.LGS_SNAPPY_COMPRESSION, 7)
    raw = batch.upload(c)
    d_file, dho, dhs, dend = tab.write_blocks(raw.buf, raw.off, raw.len, 1, 7)
    torch.cuda.synchronize()
    assert end == int(dend.cpu()[0])
    assert region == d_file[:end - 7].cpu().numpy().tobytes()
    assert np.array_equal(hoff, dho.cpu().numpy().astype(np.uint64))
    assert np.array_equal(hsize, dhs.cpu().numpy().astype(np.uint64))
    image = b"\0" * 7 + region
    res, st = tab.read_blocks_host(image, hoff, hsize, [int(x) for x in c.len])
    assert all(int(x) == tab.LGS_ST_OK for x in st)
    assert res == blocks
    # Bad handles and a damaged block in different chunks of the pipeline
    # (each chunk stages its own image): the reference's outcome for each.
    hoff2, hsize2 = hoff.copy(), hsize.copy()
    hoff2[5] = len(image) + 100                        # past the end
    hsize2[20000] = len(image)                         # runs past the end
    hoff2[40000] = len(image) - 3                      # trailer cut off
    img2 = bytearray(image)
    img2[int(hoff[65535]) + 2] ^= 0x10                 # checksum mismatch
    img2 = bytes(img2)
    res, st = tab.read_blocks_host(img2, hoff2, hsize2, [int(x) for x in c.len], True)
    for i in range(c.n):
        if i in (5, 20000, 40000, 65535):
            ost, ores = oracle.table_read_block(img2, int(hoff2[i]), int(hsize2[i]), True,
                                                int(c.len[i]))
            assert int(st[i]) == ost and res[i] == ores, i
            assert ost != tab.LGS_ST_OK, i
        else:
            assert int(st[i]) == tab.LGS_ST_OK and res[i] == blocks[i], i


def test_write_then_read_device_c2_scale(tab):
    """Size-independent property at BASELINE scale: frame 65 536 fillseq blocks
    on the device, read them back (checksums verified): identity."""
    import torch
    from lcdb_amd import batch, corpus
    c = corpus.fillseq(65536)
    raw = batch.upload(c)
    d_file, hoff, hsize, end = tab.write_blocks(raw.buf, raw.off, raw.len, 1, 0)
    torch.cuda.synchronize()
    e = int(end.cpu()[0])
    out = batch.decode_slots(c.len)
    olen, st = tab.read_blocks(d_file, e, hoff, hsize, out.buf, out.off, out.cap, out.max_cap, True)
    torch.cuda.synchronize()
    assert bool((st == 1).all())
    assert torch.equal(olen, raw.len)
    ho = batch.to_host(out)
    ho.len = olen.cpu().numpy().astype(np.uint32)
    for i in range(0, c.n, 997):
        assert ho.block(i) == c.block(i)
    # Every block's bytes: compare packed digests.
    import hashlib
    h1, h2 = hashlib.sha256(), hashlib.sha256()
    for i in range(c.n):
        h1.update(memoryview(c.block(i)))
        h2.update(memoryview(ho.block(i)))
    assert h1.digest() == h2.digest()
    # And the file region equals the oracle's framing of the first blocks.
    k = 512
    want = oracle.table_write_blocks([c.block(i) for i in range(k)], 1, 0)
    assert d_file[:want[3]].cpu().numpy().tobytes() == want[0]


_SMALL_CHUNKS = r"""
import sys
sys.path.insert(0, sys.argv[1])
import numpy as np
import oracle
from lcdb_amd import corpus, table
c = corpus.concat(corpus.fillseq(1500), corpus.random_blocks(301, 4096),
                  corpus.fillseq(7, block_size=65536))
blocks = c.blocks()
region, hoff, hsize, end = table.write_blocks_host(blocks, table.LGS_SNAPPY_COMPRESSION, 5)
assert end == 5 + len(region)
ref = oracle.table_write_blocks(blocks, 1, 5)
assert bytes(region) == ref[0], "region differs from the oracle"
assert np.array_equal(np.asarray(hoff, dtype=np.uint64), ref[1])
image = b"\0" * 5 + bytes(region)
res, st = table.read_blocks_host(image, hoff, hsize, [int(x) for x in c.len])
assert all(int(x) == table.LGS_ST_OK for x in st) and res == blocks
print("chunks ok", len(blocks))
"""


def test_host_paths_many_small_chunks(gpu, tmp_path):
    """LGS_HOST_CHUNK_MB=1 (read once at load, so in a child process): the
    table host paths run ~10 chunks through their two staging slots, an odd
    number, with 4 KiB and 64 KiB blocks; the region equals the oracle's
    framing byte for byte and every block reads back."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "small_chunks.py"
    script.write_text(_SMALL_CHUNKS)
    env = dict(os.environ, LGS_HOST_CHUNK_MB="1", PYTHONPATH=os.path.join(root, "tests"))
    r = subprocess.run([sys.executable, str(script), root], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "chunks ok 1808" in r.stdout

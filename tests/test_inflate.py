"""CPU: the dictionary reader's gzip decoder (dwpa_amd/csrc/inflate.hpp, GzipDecoder) against zlib.

help_crack hands the cracker gzip wordlists (help_crack.py:520-552).  dwpa_crack_files inflates them with its own
DEFLATE decoder (about twice zlib 1.2.11's rate on a host core, so one gz stream feeds more GPUs), which must yield
exactly the bytes zlib's gzread yields and reject what zlib rejects.  tools/bin/inflate_check decodes each file with
both, in blocks of a given size (so back-references cross block boundaries), and compares.
"""
import gzip
import os
import random
import struct
import subprocess
import zlib

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "bin", "inflate_check")


@pytest.fixture(scope="module")
def tool():
    subprocess.run(["make", "-s", "-C", ROOT, "tools/bin/inflate_check"], check=True)
    return TOOL


def _words(rng, n):
    out = []
    for i in range(n):
        if i % 7 == 0:
            out.append(bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz0123456789!@#") for _ in range(rng.randint(8, 63))))
        else:
            out.append(b"pass%08d" % rng.randrange(10 ** 8))
    return b"\n".join(out) + b"\n"


def _raw_deflate(data, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, memlevel=8):
    c = zlib.compressobj(level, zlib.DEFLATED, -15, memlevel, strategy)
    return c.compress(data) + c.flush()


def _member(data, flags=0, extra=b"", name=b"", comment=b"", hcrc=True, **kw):
    h = b"\x1f\x8b\x08" + bytes([flags]) + b"\0\0\0\0\0\xff"
    if flags & 4:
        h += struct.pack("<H", len(extra)) + extra
    if flags & 8:
        h += name + b"\0"
    if flags & 16:
        h += comment + b"\0"
    if flags & 2:
        h += struct.pack("<H", (zlib.crc32(h) & 0xFFFF) ^ (0 if hcrc else 1))
    return h + _raw_deflate(data, **kw) + struct.pack("<II", zlib.crc32(data), len(data) & 0xFFFFFFFF)


def _far_match():
    """A fixed-Huffman block whose first symbol is a match (length 3, distance 1) before any output."""
    bits = []

    def put(v, n):  # header fields and extra bits: LSB first
        bits.extend((v >> i) & 1 for i in range(n))

    def code(c, n):  # Huffman codes: MSB first
        bits.extend((c >> i) & 1 for i in range(n - 1, -1, -1))
    put(1, 1)
    put(1, 2)
    code(1, 7)  # symbol 257 (length 3)
    code(0, 5)  # distance code 0 (distance 1)
    code(0, 7)  # end of block
    bits += [0] * (-len(bits) % 8)
    return bytes(sum(b << i for i, b in enumerate(bits[k:k + 8])) for k in range(0, len(bits), 8))


def _run(tool, paths, block=None):
    args = [tool] + (["-b", str(block)] if block else []) + [str(p) for p in paths]
    r = subprocess.run(args, capture_output=True, text=True)
    lines = dict(l.split(" ", 1) for l in r.stdout.splitlines()[1:])
    return r.returncode, lines


def test_decoder_matches_zlib(tool, tmp_path):
    rng = random.Random(3)
    txt = _words(rng, 300_000)
    cases = {
        "l1.gz": gzip.compress(txt, compresslevel=1),
        "l6.gz": gzip.compress(txt, compresslevel=6),
        "l9.gz": gzip.compress(txt, compresslevel=9),
        "fixed.gz": _member(txt[:400_000], strategy=zlib.Z_FIXED),
        "huffonly.gz": _member(txt[:400_000], strategy=zlib.Z_HUFFMAN_ONLY),
        "rle.gz": _member(b"a" * 300_000 + b"ab" * 100_000 + b"abc" * 50_000 + bytes(range(256)) * 300,
                          strategy=zlib.Z_RLE),
        "stored.gz": _member(txt[:300_000], level=0),
        "random.gz": gzip.compress(rng.randbytes(2_000_000)),
        "multi.gz": gzip.compress(txt[:70_000]) + gzip.compress(b"") + gzip.compress(txt[70_000:250_000]),
        "empty.gz": gzip.compress(b""),
        "header.gz": _member(txt[:60_000], flags=2 | 4 | 8 | 16, extra=b"xyz12", name=b"words.txt",
                             comment=b"a comment"),
        "garbage.gz": gzip.compress(txt[:9_000]) + b"trailing bytes that are not gzip",
        "memlevel1.gz": _member(txt[:200_000], memlevel=1),
        "long_distance.gz": gzip.compress(rng.randbytes(40_000) + txt[:10_000] + rng.randbytes(20_000) +
                                          rng.randbytes(40_000)[:1] + txt[:10_000]),
        # compressed streams longer than the decoder's 4 MiB input buffer: stored and Huffman blocks across refills
        "big_random.gz": gzip.compress(rng.randbytes(5_000_000)),
        "big_mixed.gz": gzip.compress(b"".join(rng.randbytes(700_000) if i % 2 else (b"password%07d\n" % i) * 60_000
                                               for i in range(12)), compresslevel=1),
    }
    paths = []
    for name, blob in cases.items():
        p = tmp_path / name
        p.write_bytes(blob)
        paths.append(p)
    for block in (None, 4096, 65536 + 17):  # 4 MiB blocks, and blocks far smaller than the 32 KiB window
        rc, lines = _run(tool, paths, block)
        for p in paths:
            assert lines[str(p)].startswith("ok "), (block, p.name, lines[str(p)])
        assert rc == 0


def test_decoder_rejects_what_zlib_rejects(tool, tmp_path):
    rng = random.Random(4)
    txt = _words(rng, 40_000)
    good = gzip.compress(txt)
    bad_crc = bytearray(good)
    bad_crc[-6] ^= 1
    bad_size = bytearray(good)
    bad_size[-2] ^= 1
    body = bytearray(good)
    body[len(body) // 2] ^= 0x55
    cases = {
        "crc.gz": bytes(bad_crc),
        "isize.gz": bytes(bad_size),
        "truncated.gz": good[: len(good) // 2],
        "no_trailer.gz": good[:-8],
        "hcrc.gz": _member(txt, flags=2 | 8, name=b"n", hcrc=False),
        "corrupt.gz": bytes(body),
        "blocktype3.gz": b"\x1f\x8b\x08\0\0\0\0\0\0\xff" + bytes([0b111]) + b"\0" * 16,
        "stored_nlen.gz": b"\x1f\x8b\x08\0\0\0\0\0\0\xff" + b"\x01\x05\x00\x00\x00" + b"hello" + b"\0" * 8,
        "distance.gz": b"\x1f\x8b\x08\0\0\0\0\0\0\xff" + _far_match() + b"\0" * 8,
    }
    paths = []
    for name, blob in cases.items():
        p = tmp_path / name
        p.write_bytes(blob)
        paths.append(p)
    rc, lines = _run(tool, paths)
    for p in paths:
        res = lines[str(p)]
        assert res.startswith("error ") and not res.startswith("error none"), (p.name, res)
    assert rc == 0  # both decoders failed on every file


def _prun(tool, paths, threads=4, chunk=65536):
    r = subprocess.run([tool, "-p", str(threads), "-c", str(chunk)] + [str(p) for p in paths], capture_output=True,
                       text=True)
    return r.returncode, dict(l.split(" ", 1) for l in r.stdout.splitlines())


def test_parallel_inflate_matches_zlib(tool, tmp_path):
    """one gzip stream inflated in parallel chunks (dwpa_amd/csrc/pinflate.hpp, ParallelGunzip:
    block-boundary search, 16-bit marker phase for the unknown window, in-order marker resolution and per-member
    CRC-32/ISIZE), continued by gzread when it stops -- exactly what the dictionary reader runs.  64 KiB chunks make
    every file here dozens of chunks.  Output must equal zlib's byte for byte; the chunks must really run in parallel
    where the stream has dynamic blocks; fixed-Huffman and stored streams (no boundary to find) still decode, in one
    piece."""
    rng = random.Random(13)
    txt = _words(rng, 200_000)
    rnd_words = b"\n".join(bytes(rng.randint(0x21, 0x7E) for _ in range(rng.randint(8, 20)))
                           for _ in range(150_000)) + b"\n"
    cases = {
        "rand_l1.gz": gzip.compress(rnd_words, compresslevel=1),
        "text_l6.gz": gzip.compress(txt, compresslevel=6),
        "text_l9.gz": gzip.compress(txt, compresslevel=9),
        "huffonly.gz": _member(txt, strategy=zlib.Z_HUFFMAN_ONLY),
        "rle.gz": _member(b"a" * 300_000 + txt[:600_000] + b"ab" * 100_000, strategy=zlib.Z_RLE),
        "fixed.gz": _member(txt[:600_000], strategy=zlib.Z_FIXED),
        "stored.gz": _member(txt[:600_000], level=0),
        "mixed.gz": gzip.compress(txt[:300_000] + rng.randbytes(400_000) + txt[300_000:700_000], compresslevel=1),
        "multi.gz": gzip.compress(txt[:500_000]) + gzip.compress(b"") + gzip.compress(rnd_words[:700_000], 1) +
                    gzip.compress(txt[500_000:]),
        "garbage.gz": gzip.compress(txt, compresslevel=1) + b"trailing bytes that are not gzip" * 50,
    }
    paths = []
    for name, blob in cases.items():
        p = tmp_path / name
        p.write_bytes(blob)
        paths.append(p)
    for threads in (1, 3, 8):
        rc, lines = _prun(tool, paths, threads)
        for p in paths:
            assert lines[str(p)].startswith("ok "), (threads, p.name, lines[str(p)])
        assert rc == 0
    info = {p.name: lines[str(p)].split() for p in paths}
    par = {k: int(v[v.index("parallel") + 1]) for k, v in info.items()}
    chunks = {k: int(v[v.index("chunks") + 1]) for k, v in info.items()}
    for k in ("rand_l1.gz", "text_l6.gz", "text_l9.gz", "huffonly.gz", "multi.gz"):
        assert par[k] >= chunks[k] // 2 and par[k] >= 4, (k, par[k], chunks[k])
    assert par["fixed.gz"] == 1 and par["stored.gz"] == 1
    assert all(v[v.index("stop") + 1] == "none" for k, v in info.items()), info


def test_parallel_inflate_false_boundary_falls_back(tool, tmp_path):
    """A boundary search can find a position that starts a perfectly valid dynamic block which is not a block of this
    stream: here stored blocks carry the raw bytes of another deflate stream, so the search in later chunks finds
    that nested stream's blocks.  The chunk before it must then fail to land on the find, the parallel decode stop
    at that point, and gzread continue: the output is still exactly zlib's and the stop reason is a boundary
    mismatch, not damage."""
    rng = random.Random(15)
    txt = _words(rng, 120_000)
    nested = _raw_deflate(txt, level=6)
    plain = gzip.compress(txt[:200_000], compresslevel=6)
    cases = {
        # stored blocks only: every find is false, chunk 0 runs into the first one
        "stored_nested.gz": _member(txt[:100_000] + nested + txt[:50_000], level=0),
        # a real dynamic stream, then a stored member whose payload is another stream's deflate bytes
        "mixed_nested.gz": plain + _member(nested + txt[:30_000], level=0),
    }
    paths = []
    for name, blob in cases.items():
        p = tmp_path / name
        p.write_bytes(blob)
        paths.append(p)
    for threads in (1, 4):
        rc, lines = _prun(tool, paths, threads)
        for p in paths:
            assert lines[str(p)].startswith("ok "), (threads, p.name, lines[str(p)])
        assert rc == 0
        stops = {p.name: lines[str(p)].split(" stop ", 1)[1] for p in paths}
        assert stops["stored_nested.gz"] != "none", stops  # the nested blocks were found and rejected
        for reason in stops.values():
            assert reason == "none" or "boundary" in reason or "chunk" in reason, stops


def test_parallel_inflate_damaged_like_gzread(tool, tmp_path):
    """Damage inside a parallel decode: a cut stream yields exactly gzread's bytes (the reader hands over to gzread
    after what was delivered); a corrupt trailer or body yields at least gzread's bytes and fails."""
    rng = random.Random(14)
    good = gzip.compress(_words(rng, 200_000), compresslevel=6)
    body = bytearray(good)
    body[len(body) * 3 // 4] ^= 0x55
    crc = bytearray(good)
    crc[-6] ^= 1
    cases = {"cut_mid.gz": good[: len(good) // 2], "cut_end.gz": good[:-3], "cut_trailer.gz": good[:-8],
             "crc.gz": bytes(crc), "corrupt.gz": bytes(body)}
    paths = []
    for name, blob in cases.items():
        p = tmp_path / name
        p.write_bytes(blob)
        paths.append(p)
    rc, lines = _prun(tool, paths, 4)
    for p in paths:
        assert lines[str(p)].startswith("error both"), (p.name, lines[str(p)])
    assert rc == 0


def test_parallel_inflate_under_thread_sanitizer(tmp_path):
    """The parallel inflate's threads -- the pread loader (round 4: it replaced the mmap, which raised SIGBUS when a
    dictionary was rewritten while read), the boundary-search / decode workers and the joining reader -- under
    ThreadSanitizer (tools/bin/inflate_check_tsan): no data race reported, output still equal to zlib's, on an
    intact and on a cut stream.  The sanitizer build loads in 16 KiB steps, so the boundary probes (which decode whole
    candidate blocks past their chunk) keep reaching bytes still being loaded: ADVICE r4, a probe reads only what the
    loader has published and waits for more when it gets there."""
    subprocess.run(["make", "-s", "-C", ROOT, "tools/bin/inflate_check_tsan"], check=True)
    tsan = os.path.join(ROOT, "tools", "bin", "inflate_check_tsan")
    rng = random.Random(16)
    good = gzip.compress(_words(rng, 150_000), compresslevel=6)
    (tmp_path / "good.gz").write_bytes(good)
    (tmp_path / "cut.gz").write_bytes(good[: len(good) * 2 // 3])
    r = subprocess.run([tsan, "-p", "8", "-c", "65536", str(tmp_path / "good.gz"), str(tmp_path / "cut.gz")],
                       capture_output=True, text=True, timeout=600)
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-3000:]
    lines = dict(l.split(" ", 1) for l in r.stdout.splitlines())
    assert lines[str(tmp_path / "good.gz")].startswith("ok "), lines
    assert lines[str(tmp_path / "cut.gz")].startswith("error both"), lines

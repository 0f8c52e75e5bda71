"""CPU: the dwpa_crack_files dictionary reader (dwpa_amd/csrc/dict_reader.hpp) yields exactly the words of the
wordlists help_crack hands to the cracker (help_crack.py:520-552; maint.php:55-60 writes $HEX[] for
non-printable words): one word per line, "\\n" or "\\r\\n", empty lines kept (the 8..63 filter drops them later), a
last line without "\\n" still a word, $HEX[..] decoded as hc_unhex does (web/common.php:3-25).

The reader runs as an inflate thread feeding a line-cutting thread; the large gzip file here makes lines straddle
the 4 MiB inflate blocks.  tools/bin/inflate_bench --dump prints the words it yields.
"""
import gzip
import os
import random
import subprocess

import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "bin", "inflate_bench")


def _expected(blobs):
    out = []
    for data in blobs:
        parts = data.split(b"\n")
        if parts[-1] == b"":
            parts.pop()
        for w in parts:
            if w.endswith(b"\r"):
                w = w[:-1]
            out.append(O.hc_unhex(w) if len(w) > 5 else w)
    return out


def test_reader_words_match(tmp_path):
    subprocess.run(["make", "-s", "-C", ROOT, "tools/bin/inflate_bench"], check=True)
    rng = random.Random(61)
    small = (b"password\r\n\r\n$HEX[41424344]\n$HEX[4142zz]\n$HEX[]\n$HEX[\nplain word\n" +
             b"$HEX[" + bytes(range(1, 40)).hex().encode() + b"]\r\nx" * 3 + b"last-without-newline")
    big_words = [bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz0123456789!@") for _ in range(rng.randint(1, 30)))
                 for _ in range(400_000)]
    big = b"\n".join(big_words) + b"\n"
    files = []
    for name, data, gz in (("a.txt", small, False), ("b.txt.gz", big, True), ("c.txt", b"", False),
                           ("d.txt.gz", b"tail\r\nno-newline-at-end", True)):
        path = tmp_path / name
        if gz:
            with gzip.open(path, "wb", compresslevel=1) as f:
                f.write(data)
        else:
            path.write_bytes(data)
        files.append((str(path), data))
    r = subprocess.run([TOOL, "--dump"] + [p for p, _ in files], capture_output=True, check=True)
    got = [bytes.fromhex(l) for l in r.stdout.decode().split("\n")[:-1]]
    exp = _expected([d for _, d in files])
    assert len(got) == len(exp)
    assert got == exp


def _parse_passes(stdout):
    """inflate_bench --passes output -> ([[cache_hits, words]] per pass, [file statuses] per pass); the cache's entry
    count per pass is in _parse_passes.entries."""
    out, status, cur = [], [], None
    entries = _parse_passes.entries = []
    for line in stdout.decode().split("\n")[:-1]:
        if line.startswith("#pass"):
            cur = [int(line.split()[3]), []]
            out.append(cur)
            entries.append(int(line.split()[5]))
        elif line.startswith("#status"):
            status.append([int(x) for x in line.split()[1:]])
        else:
            cur[1].append(bytes.fromhex(line))
    return out, status


def test_reader_cache_replays_same_words(tmp_path):
    """crack_files' ChunkSource keeps each dictionary it read to the end in the process-wide DictCache
    (dict_reader.hpp) and replays it on the next work unit: the second and third passes over the same files yield
    exactly the words of the first and the cache reports one hit per file and pass; DWPA_DICT_CACHE_MB=0 turns it
    off."""
    subprocess.run(["make", "-s", "-C", ROOT, "tools/bin/inflate_bench"], check=True)
    rng = random.Random(62)
    files = []
    for k in range(3):
        words = [bytes(rng.choice(b"abcdefghij0123456789") for _ in range(rng.randint(0, 20))) for _ in range(30_000)]
        data = b"\n".join(words) + (b"\n" if k != 1 else b"")
        path = tmp_path / ("w%d.txt.gz" % k)
        with gzip.open(path, "wb", compresslevel=1) as f:
            f.write(data)
        files.append((str(path), data))

    def passes(k, env=None):
        r = subprocess.run([TOOL, "--passes", str(k)] + [p for p, _ in files], capture_output=True, check=True,
                           env=env)
        return _parse_passes(r.stdout)[0]

    exp = sorted(_expected([d for _, d in files]))
    got = passes(3)
    assert [h for h, _ in got] == [0, 3, 6]
    for _, words in got:
        assert sorted(words) == exp
    off = passes(2, env=dict(os.environ, DWPA_DICT_CACHE_MB="0"))
    assert [h for h, _ in off] == [0, 0] and all(sorted(w) == exp for _, w in off)


PARALLEL = dict(os.environ, DWPA_INFLATE_CHUNK_MB="1", DWPA_INFLATE_THREADS="4")  # ParallelGunzip from 4 MiB up


@pytest.mark.parametrize("env", [None, PARALLEL], ids=["single", "parallel"])
def test_damaged_gzip_scanned_to_the_damage_like_gzread(tmp_path, env):
    """a cut download must not fail the work unit forever.  hashcat reads wordlists through
    zlib's gzread, which delivers every byte decodable before the cut and then reports end of file; the crack
    path's reader (ChunkSource, the same code dwpa_crack_files runs) now yields exactly those words, flags the file
    as damaged (status 1) and keeps going with the next file; a damaged file is never cached, and an intact file
    next to it still is.  A CRC-corrupted trailer (a data error): gzread drops the read the error lands in, so the
    words are a prefix of the file's, and the file is damaged.  A cut inside the first 4 MiB block and one
    far past it (the reader's own decoder hands over to zlib at the failing block)."""
    import zlib
    subprocess.run(["make", "-s", "-C", ROOT, "tools/bin/inflate_bench"], check=True)
    rng = random.Random(63)
    words = [bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz0123456789") for _ in range(rng.randint(4, 24)))
             for _ in range(900_000)]
    data = b"\n".join(words) + b"\n"
    full = gzip.compress(data, compresslevel=6)
    good_words = [b"intact-%d" % i for i in range(1000)]
    good = tmp_path / "good.txt.gz"
    good.write_bytes(gzip.compress(b"\n".join(good_words) + b"\n"))
    cases = {"cut_early": full[:len(full) // 7], "cut_late": full[:len(full) - 5000],
             "bad_crc": full[:-8] + bytes([full[-8] ^ 0xFF]) + full[-7:]}
    for name, blob in cases.items():
        bad = tmp_path / (name + ".txt.gz")
        bad.write_bytes(blob)
        r = subprocess.run([TOOL, "--passes", "2", str(bad), str(good)], capture_output=True, check=True, env=env)
        passes, status = _parse_passes(r.stdout)
        assert status == [[1, 0], [1, 0]], name
        assert [h for h, _ in passes] == [0, 1], name  # only the intact file is replayed from the cache
        for _, got in passes:
            mine = [w for w in got if not w.startswith(b"intact-")]
            assert sorted(w for w in got if w.startswith(b"intact-")) == sorted(good_words)
            if name == "bad_crc":
                # a data error loses gzread's failing read (the parallel decoder keeps it): a prefix of the words
                # (the last one may be cut)
                assert 0 < len(mine) <= len(words), name
                assert mine[:-1] == words[:len(mine) - 1] and words[len(mine) - 1].startswith(mine[-1])
            else:
                exp_text = zlib.decompressobj(31).decompress(blob)  # everything inflate yields before the cut
                assert 0 < len(exp_text) < len(data)
                assert mine == _expected([exp_text]), name


def test_cache_drops_stale_entry_of_a_changed_file(tmp_path):
    """a dictionary re-downloaded under the same path (new size/mtime/inode) must not leave its old decode
    in the DictCache until LRU eviction: the next read drops the stale entry and caches the new file, so the cache
    keeps one entry per path and every pass yields the file's current words."""
    subprocess.run(["make", "-s", "-C", ROOT, "tools/bin/inflate_bench"], check=True)
    p = tmp_path / "cracked.txt"
    p.write_bytes(b"".join(b"word%05d\n" % i for i in range(5000)))
    r = subprocess.run([TOOL, "--passes", "3", str(p)], capture_output=True, check=True,
                       env=dict(os.environ, DWPA_TEST_REWRITE=str(p)))
    passes, status = _parse_passes(r.stdout)
    assert [h for h, _ in passes] == [0, 0, 0]  # every pass sees a changed file: no stale replay
    assert _parse_passes.entries == [1, 1, 1]
    for k, (_, words) in enumerate(passes):
        assert words[-1] == (b"word04999" if k == 0 else b"added-after-pass-%d" % (k - 1))
        assert len(words) == 5000 + k


def test_item_queue_covers_every_word_and_balances_workers(tmp_path):
    """The crack path's work items (ItemQueue over ChunkSource, dict_reader.hpp) with 1, 3 and 8 shard workers
    pulling concurrently (tools/bin/item_queue_check, each worker holding an item for a time proportional to its
    size, as a device scanning it): every word of a plain and a gzip dictionary is handed out exactly once, and with
    several workers no worker ends up with more than twice the mean (the pre-round-3 doubling items gave one of 8
    workers 4.6x the mean on a 20M-word dictionary, profiles/r03/crack_balance/)."""
    subprocess.run(["make", "-s", "-C", ROOT, "tools/bin/item_queue_check"], check=True)
    tool = os.path.join(ROOT, "tools", "bin", "item_queue_check")
    n = 600_000
    plain = tmp_path / "w.txt"
    plain.write_bytes(b"".join(b"w%07d\n" % i for i in range(n)))
    gz = tmp_path / "w.txt.gz"
    gz.write_bytes(gzip.compress(plain.read_bytes(), compresslevel=6))
    import json
    for path in (plain, gz):
        for workers in (1, 3, 8):
            r = subprocess.run([tool, str(workers), "4096", "131072", "400000", str(path)], capture_output=True,
                               text=True, timeout=120)
            assert r.returncode == 0, r.stderr
            d = json.loads(r.stdout)
            assert d["words_total"] == n and d["unique"] and not d["io_error"], (path.name, workers, d)
            w = [x["words"] for x in d["workers"]]
            if workers > 1 and path == plain:
                assert max(w) <= 2 * n / workers, (workers, w)


def test_reader_caps_overlong_lines(tmp_path):
    """A line longer than the reader's 1 MiB cap (binary garbage without a '\\n', a runaway line) is still one word,
    kept to its first MiB -- every consumer rejects a word that long -- and the next line comes through intact, in
    plain and gzip files, across the 4 MiB inflate blocks."""
    subprocess.run(["make", "-s", "-C", ROOT, "tools/bin/inflate_bench"], check=True)
    cap = 1 << 20
    hexline = b"$HEX[" + b"41" * (3 * cap) + b"]"
    data = b"first\n" + b"\x00" * (5 * cap) + b"\nnext\r\n" + hexline + b"\nlast"
    plain, gz = tmp_path / "long.txt", tmp_path / "long.txt.gz"
    plain.write_bytes(data)
    with gzip.open(gz, "wb", compresslevel=1) as f:
        f.write(data)
    r = subprocess.run([TOOL, "--dump", str(plain), str(gz)], capture_output=True, check=True)
    got = [bytes.fromhex(l) for l in r.stdout.decode().split("\n")[:-1]]
    one = [b"first", b"\x00" * cap, b"next", hexline[:cap], b"last"]
    assert got == one + one


def test_reader_threads_never_abort_on_long_lines(tmp_path):
    """the crack path's reader threads (ChunkSource, the inflater) run no exception out of their
    thread -- std::terminate would end the caller's process (a PHP-FPM worker, help_crack).  A gzip dictionary of
    1 MiB lines made the chunk reserve ask for words x 1 MiB (now capped), and an allocation that fails inside a
    reader thread now fails the call like an I/O error.  Under a 16 GiB address-space cap every line comes through;
    under 600 and 300 MiB the tool must still exit 0 (io_error), never abort (SIGABRT, -6)."""
    import gzip
    import json
    import resource
    subprocess.run(["make", "-s", "-C", ROOT, "tools/bin/item_queue_check"], check=True)
    tool = os.path.join(ROOT, "tools", "bin", "item_queue_check")
    path = tmp_path / "long.txt.gz"
    with gzip.open(path, "wb", compresslevel=1) as f:
        for i in range(300):
            f.write(bytes([97 + i % 26]) * (1 << 20) + b"\n")
    env = dict(os.environ, MALLOC_ARENA_MAX="2")  # glibc's per-thread arenas reserve address space too
    for cap, whole in ((16 << 30, True), (600 << 20, False), (300 << 20, False)):
        def limit(c=cap):
            resource.setrlimit(resource.RLIMIT_AS, (c, c))
        r = subprocess.run([tool, "2", "64", "1024", "0", str(path)], capture_output=True, text=True,
                           preexec_fn=limit, timeout=300, env=env)
        assert r.returncode == 0, (cap, r.returncode, r.stderr[-500:])
        out = json.loads(r.stdout)
        if whole:
            assert out["words_total"] == 300 and not out["io_error"]
        else:  # the library reports the failed allocation (or the tool's own copies ran out first)
            assert out["io_error"] or out["tool_oom"] or out["words_total"] == 300

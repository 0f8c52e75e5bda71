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
        out, cur = [], None
        for line in r.stdout.decode().split("\n")[:-1]:
            if line.startswith("#pass"):
                cur = [int(line.split()[3]), []]
                out.append(cur)
            else:
                cur[1].append(bytes.fromhex(line))
        return out

    exp = sorted(_expected([d for _, d in files]))
    got = passes(3)
    assert [h for h, _ in got] == [0, 3, 6]
    for _, words in got:
        assert sorted(words) == exp
    off = passes(2, env=dict(os.environ, DWPA_DICT_CACHE_MB="0"))
    assert [h for h, _ in off] == [0, 0] and all(sorted(w) == exp for _, w in off)

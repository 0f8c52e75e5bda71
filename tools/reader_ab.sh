#!/bin/bash
# Dictionary-reader A/B on this host: tools/bin/inflate_bench over two 200 MB gzip wordlists -- C2-shaped random
# printable words (what bench.py --workload c2files writes, mostly literals) and a word-list-like file (digits and
# repeated stems, mostly matches) -- with the reader on GzipDecoder and on zlib's gzread (DWPA_INFLATE=zlib).
# Output: one JSON line per (file, inflater) in $OUT.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/reader_ab}
mkdir -p $OUT
TMP=$(mktemp -d)
trap 'rm -rf $TMP' EXIT
python3 - "$TMP" <<'PY'
import gzip, sys
import numpy as np
tmp = sys.argv[1]
rng = np.random.default_rng(7)
n = 17_000_000
lens = np.clip(rng.geometric(0.3, n) + 7, 8, 63)
ends = np.cumsum(lens + 1)
text = rng.integers(0x21, 0x7F, int(ends[-1]), dtype=np.uint8)
text[ends - 1] = 0x0A
with gzip.open(f"{tmp}/c2.txt.gz", "wb", compresslevel=1) as f:
    f.write(text.tobytes())
stems = [b"password", b"qwerty", b"dragon", b"monkey", b"letmein", b"sunshine", b"princess", b"football"]
words = [stems[i % 8] + b"%d" % v for i, v in enumerate(rng.integers(0, 10 ** 7, 20_000_000))]
with gzip.open(f"{tmp}/list.txt.gz", "wb", compresslevel=6) as f:
    f.write(b"\n".join(words) + b"\n")
PY
for f in c2 list; do
  for t in ${THREADS:-1 4 8 12}; do
    DWPA_INFLATE_THREADS=$t timeout -k 10 120 tools/bin/inflate_bench $TMP/$f.txt.gz > $OUT/${f}_t$t.json
  done
  DWPA_INFLATE=zlib timeout -k 10 120 tools/bin/inflate_bench $TMP/$f.txt.gz > $OUT/${f}_zlib.json
  timeout -k 10 120 tools/bin/inflate_check -r 2 $TMP/$f.txt.gz > $OUT/${f}_check.txt
  for t in 4 8 12; do
    timeout -k 10 120 tools/bin/inflate_check -r 2 -p $t $TMP/$f.txt.gz > $OUT/${f}_pcheck_t$t.txt
  done
done
cat $OUT/*.json

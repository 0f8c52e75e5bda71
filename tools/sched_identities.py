"""XOR-type ops of the SHA-1 message schedule for the PBKDF2 loop's 84-byte message (W0..W4 variable,
W5 = 0x80000000, W6..W14 = 0, W15 = 672) when W[t] may use the recurrence applied 2^j times:
W[t] = rotl(W[t-3s] ^ W[t-8s] ^ W[t-14s] ^ W[t-16s], s), s = 2^j, t >= 16s.  A 3-input XOR takes two more terms,
the folded constant counts as one term.  python3 tools/sched_identities.py -> per max-j totals and the t that change
(crypto_dev.hpp sched_w; profiles/r05/sched_identities/)."""
KIND = ["v"] * 5 + ["c"] + ["z"] * 9 + ["c"]


def cost(terms):
    nv = sum(1 for k in terms if k == "v")
    n = nv + (1 if "c" in terms else 0)
    return 0 if nv == 0 else n // 2


def schedule(max_j):
    k, total, forms = KIND[:], 0, {}
    for t in range(16, 80):
        best = (cost([k[t - 3], k[t - 8], k[t - 14], k[t - 16]]), 0)
        for j in range(1, max_j + 1):
            s = 1 << j
            if t >= 16 * s:
                best = min(best, (cost([k[t - 3 * s], k[t - 8 * s], k[t - 14 * s], k[t - 16 * s]]), j))
        total += best[0]
        if best[1]:
            forms[t] = best[1]
        k.append("v")
    return total, forms


if __name__ == "__main__":
    for j in (0, 1, 2):
        total, forms = schedule(j)
        print(f"max j = {j}: {total} XOR-type ops per compression; t using j > 0: {sorted(forms)}")

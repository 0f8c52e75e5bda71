"""CPU: the SHA-1 schedule identities the PBKDF2 loop uses (crypto_dev.hpp sched_w).

For t >= 16 * 2^j the recurrence applied 2^j times gives W[t] = rotl(W[t-3s] ^ W[t-8s] ^ W[t-14s] ^ W[t-16s], s)
with s = 2^j.  Checked here on random messages of the kernels' two layouts (the 84-byte HMAC message and a key pad
block), against the schedule computed by its definition; and the XOR-op counts the kernel's form choice is priced
on (tools/sched_identities.py).  The GPU parity tests hold the compiled kernels to the oracle end to end."""
import random

from tools import sched_identities as SI


def rotl(x, n):
    return ((x << n) | (x >> (32 - n))) & 0xFFFFFFFF


def schedule(w16):
    w = list(w16)
    for t in range(16, 80):
        w.append(rotl(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1))
    return w


def test_identities_hold_on_both_layouts():
    rng = random.Random(5)
    for _ in range(200):
        u = [rng.getrandbits(32) for _ in range(5)]
        msg84 = u + [0x80000000] + [0] * 9 + [672]
        key = [rng.getrandbits(32) ^ 0x36363636 for _ in range(4)] + [0x36363636] * 12
        anything = [rng.getrandbits(32) for _ in range(16)]
        for m in (msg84, key, anything):
            w = schedule(m)
            for j in (1, 2):
                s = 1 << j
                for t in range(16 * s, 80):
                    assert w[t] == rotl(w[t - 3 * s] ^ w[t - 8 * s] ^ w[t - 14 * s] ^ w[t - 16 * s], s), (t, j)


def test_xor_counts_of_the_84_byte_message():
    assert SI.schedule(0)[0] == 112  # the plain recurrence (rounds 1-4; C_min 1,878.5)
    assert SI.schedule(1)[0] == 99   # j <= 1: the lone-wave kernels
    total, forms = SI.schedule(2)
    assert total == 84                # j <= 2: tools/cmin.py prices C_min on this (1,822.5)
    assert sorted(t for t, j in forms.items() if j == 1) == list(range(34, 47))
    assert sorted(t for t, j in forms.items() if j == 2) == list(range(64, 79))


def test_issue_cost_floor():
    from tools.cmin import c_min
    assert c_min() == 1822.5                   # the cheapest known compression (84 schedule XORs)
    assert c_min(sched_xors=99) == 1852.5      # j <= 1
    assert c_min(sched_xors=112) == 1878.5     # the plain recurrence, rounds 1-4

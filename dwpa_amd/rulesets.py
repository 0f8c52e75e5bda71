"""Rule sets for bench.py and the tests (the reference's file itself stays in the reference).

wpa_rules(): a WPA-oriented hashcat rule set composed from the 16 ops dwpa's bestWPA.rule uses
(`: r u l c T0 $X ^X ] [ sXY DN 'N d pN f`, help_crack/bestWPA.rule), with a similar op mix: suffix digits and
years, truncate-then-append, prefixes, leetspeak, duplication/reflection.  Used by bench.py's rule-amplified
config and by the tests (the reference's file itself stays in the reference)."""


def wpa_rules() -> list:
    r = [":", "r", "u", "l", "c", "T0"]
    for d in "0123456789":
        r += [f"${d}", f"] ${d}"]
    for a, b in [("1", "2"), ("2", "1"), ("6", "9"), ("0", "7"), ("8", "8")]:
        r += [f"${a} ${b}", f"] ${a} ${b}", f"] ] ${a} ${b}", f"^{b} ^{a}"]
    for s in ["123", "1234", "2020", "2021", "2022", "2023", "2024", "007"]:
        app = " ".join(f"${c}" for c in s)
        r += [app, "] " + app, "] ] " + app, "^" + " ^".join(reversed(s))]
    r += ["]", "] ]", "] ] ]", "] ] ] ]"]
    r += [f"^{d}" for d in "0123456789"]
    r += ["^e ^h ^t", "sa@ sc< se3 si1 so0 ss$", "sa4 se3 so0", "si! so0"]
    for c in "!*#@$.":
        r += [f"${c}", f"] ${c}", f"^{c}", f"^{c} ${c}"]
    r += ["$@ $1", "] $@ $1", "$@ $1 $2 $3", "$@ $2 $0 $2 $4"]
    r += ["[", "[ [", "[ [ [", "D2", "D3", "D4", "'3 d", "'4 d", "'2 p2", "'3 p2", "'4 p2", "'3 f", "'4 f"]
    r += ["c $1", "c $!", "u $1", "c $1 $2 $3", "r $1", "d", "f", "p1", "T0 $1", "T1", "T2 T3"]
    return r


def server_rules() -> list:
    """wpa_rules() plus the kind of lines an operator adds to a dictionary's `dicts.rules` (db/wpa.sql:48,
    INSTALL.md:110), which get_work merges (web/content/get_work.php:86-92) and help_crack runs with `-S -r`
    (help_crack.py:931-933): title case, inserts and overwrites, block duplication, toggles after separators, byte
    arithmetic, swaps, memory and reject functions of hashcat's rule language."""
    r = wpa_rules()
    r += ["E", "E $1", "E $!", "e- $1", "e_", "30 ", "30-", "30_ 31_", "E @ ", "E @-"]
    r += [f"i{p}{c}" for p in "0245" for c in "-_."] + ["o0P", "o0p $1", "i1@ i3@", "x04 $2 $0 $2 $4", "x05 d",
                                                      "O02", "O13 $1", "*01", "*23 *45", "k", "K", "k K $1"]
    r += ["y2", "Y2", "y3 $1", "Y3 ^1", "z2", "Z2 $!", "+0", "-0", "+0 +1", ".0", ",1", "L0", "R0 $1"]
    r += ["M l 4", "M u 6", "M r 4", "M c $1 4", "u M l X002", "M $- 4", "l M u Q", "M Q", "r Q", "M r Q $9"]
    r += [">8 <G", ">9 $1", "<8 $1 $2 $3", "_8 $1", "/a sa4", "!a $a", "(a $1", ")1 $2", "=1a o14", "%2a sa@"]
    return r

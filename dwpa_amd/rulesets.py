"""A WPA-oriented hashcat rule set composed from the 16 ops dwpa's bestWPA.rule uses
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

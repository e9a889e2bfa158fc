#!/usr/bin/env python3
"""Generates odigos_amd/csrc/unicode_tables.cpp: the Unicode data the DFA
compiler (regex_dfa.cpp) needs for Go regexp's \\p{..} classes and (?i)
folding of non-ASCII runes.

Source data (no network here): the image's ICU 70 (libicuuc.so.70,
Unicode 14.0.0, through ctypes) for the general categories, the Script
property and the simple case mappings; the `regex` module (its own, newer
Unicode) only for scripts ICU 70 does not know (Kawi, Nag_Mundari: 15.0).
Without ICU: Python's unicodedata (13.0.0) and the `regex` module, as
before round 4.  Go 1.25's unicode package is Unicode 15.0.0: code points
assigned in 15.0 are parity unpinned.

Run: python3 tools/gen_unicode_tables.py > odigos_amd/csrc/unicode_tables.cpp
     python3 tools/gen_unicode_tables.py --c > oracle/unicode_data.c   (the oracle's own copy)
"""
import ctypes as C
import sys
import unicodedata

import regex

ICU_PATH = "/usr/lib/x86_64-linux-gnu/libicuuc.so.70"
# UCharCategory (uchar.h) -> Go / Unicode two-letter names; 0 is unassigned
ICU_CATS = [None, "Lu", "Ll", "Lt", "Lm", "Lo", "Mn", "Me", "Mc", "Nd", "Nl", "No", "Zs", "Zl", "Zp", "Cc", "Cf",
            "Co", "Cs", "Pd", "Ps", "Pe", "Pc", "Po", "Sm", "Sc", "Sk", "So", "Pi", "Pf"]


class Icu:
    def __init__(self, path=ICU_PATH, ver=70):
        L = C.CDLL(path)
        def fn(name, res, args):
            f = getattr(L, "%s_%d" % (name, ver))
            f.restype, f.argtypes = res, args
            return f
        self.char_type = fn("u_charType", C.c_int8, [C.c_int32])
        self.get_script = fn("uscript_getScript", C.c_int, [C.c_int32, C.POINTER(C.c_int)])
        self.script_name = fn("uscript_getName", C.c_char_p, [C.c_int])
        self.tolower = fn("u_tolower", C.c_int32, [C.c_int32])
        self.toupper = fn("u_toupper", C.c_int32, [C.c_int32])
        self.totitle = fn("u_totitle", C.c_int32, [C.c_int32])
        self.fold = fn("u_foldCase", C.c_int32, [C.c_int32, C.c_uint32])
        v = (C.c_uint8 * 4)()
        fn("u_getUnicodeVersion", None, [C.POINTER(C.c_uint8)])(v)
        self.version = "%d.%d.%d" % (v[0], v[1], v[2])

    def script(self, c):
        e = C.c_int(0)
        return self.script_name(self.get_script(c, C.byref(e))).decode()


def load_icu():
    try:
        return Icu()
    except (OSError, AttributeError):
        return None

MAX = 0x10FFFF
CATS = ["Cc", "Cf", "Co", "Cs", "Ll", "Lm", "Lo", "Lt", "Lu", "Mc", "Me", "Mn", "Nd", "Nl", "No", "Pc", "Pd", "Pe",
        "Pf", "Pi", "Po", "Ps", "Sc", "Sk", "Sm", "So", "Zl", "Zp", "Zs"]
# unicode.Scripts of Go 1.25 (Unicode 15.0.0 script names)
SCRIPTS = """Adlam Ahom Anatolian_Hieroglyphs Arabic Armenian Avestan Balinese Bamum Bassa_Vah Batak Bengali Bhaiksuki
Bopomofo Brahmi Braille Buginese Buhid Canadian_Aboriginal Carian Caucasian_Albanian Chakma Cham Cherokee Chorasmian
Common Coptic Cuneiform Cypriot Cypro_Minoan Cyrillic Deseret Devanagari Dives_Akuru Dogra Duployan
Egyptian_Hieroglyphs Elbasan Elymaic Ethiopic Georgian Glagolitic Gothic Grantha Greek Gujarati Gunjala_Gondi Gurmukhi
Han Hangul Hanifi_Rohingya Hanunoo Hatran Hebrew Hiragana Imperial_Aramaic Inherited Inscriptional_Pahlavi
Inscriptional_Parthian Javanese Kaithi Kannada Katakana Kawi Kayah_Li Kharoshthi Khitan_Small_Script Khmer Khojki
Khudawadi Lao Latin Lepcha Limbu Linear_A Linear_B Lisu Lycian Lydian Mahajani Makasar Malayalam Mandaic Manichaean
Marchen Masaram_Gondi Medefaidrin Meetei_Mayek Mende_Kikakui Meroitic_Cursive Meroitic_Hieroglyphs Miao Modi Mongolian
Mro Multani Myanmar Nabataean Nag_Mundari Nandinagari New_Tai_Lue Newa Nko Nushu Nyiakeng_Puachue_Hmong Ogham Ol_Chiki
Old_Hungarian Old_Italic Old_North_Arabian Old_Permic Old_Persian Old_Sogdian Old_South_Arabian Old_Turkic Old_Uyghur
Oriya Osage Osmanya Pahawh_Hmong Palmyrene Pau_Cin_Hau Phags_Pa Phoenician Psalter_Pahlavi Rejang Runic Samaritan
Saurashtra Sharada Shavian Siddham SignWriting Sinhala Sogdian Sora_Sompeng Soyombo Sundanese Syloti_Nagri Syriac
Tagalog Tagbanwa Tai_Le Tai_Tham Tai_Viet Takri Tamil Tangsa Tangut Telugu Thaana Thai Tibetan Tifinagh Tirhuta Toto
Ugaritic Vai Vithkuqi Wancho Warang_Citi Yezidi Yi Zanabazar_Square""".split()


def ranges(cps):
    out, lo, prev = [], None, None
    for c in cps:
        if lo is None:
            lo = prev = c
        elif c == prev + 1:
            prev = c
        else:
            out.append((lo, prev))
            lo = prev = c
    if lo is not None:
        out.append((lo, prev))
    return out


def main():
    icu = None if "--no-icu" in sys.argv else load_icu()
    version = icu.version if icu else unicodedata.unidata_version
    cat_of = {}
    for c in range(MAX + 1):
        g = ICU_CATS[icu.char_type(c)] if icu else unicodedata.category(chr(c))
        if g is not None and g != "Cn":
            cat_of[c] = g
    assigned = sorted(cat_of)
    tables = {}
    for g in CATS:
        tables[g] = ranges([c for c in assigned if cat_of[c] == g])
    # the whole-range string for the regex module (surrogates cannot be encoded)
    text = "".join(chr(c) for c in range(MAX + 1) if not 0xD800 <= c <= 0xDFFF)
    base = [c for c in range(MAX + 1) if not 0xD800 <= c <= 0xDFFF]
    scripts = {}
    aset = set(assigned)
    icu_sc = {}
    if icu:
        for c in range(MAX + 1):
            if 0xD800 <= c <= 0xDFFF:
                continue
            icu_sc.setdefault(icu.script(c), []).append(c)
    for s in SCRIPTS:
        if s in icu_sc:
            scripts[s] = ranges([c for c in icu_sc[s] if c in aset or s in ("Common", "Inherited")])
            continue
        pat = regex.compile(r"\p{Script=%s}" % s)
        cps = [base[m.start()] for m in pat.finditer(text)]
        mine = [c for c in cps if c in aset]
        scripts[s] = ranges(mine if mine else cps)
    # simple case folding orbits: single-rune lower / upper / casefold
    # mappings joined into classes; the Turkic dotted / dotless i (CaseFolding
    # status T, not part of simple folding) stay alone
    parent = {}

    def find(x):
        while parent.get(x, x) != x:
            parent[x] = parent.get(parent[x], parent[x])
            x = parent[x]
        return x

    def union(a, b):
        ra, rb = find(a), find(b)
        if ra != rb:
            parent[max(ra, rb)] = min(ra, rb)

    for c in assigned:
        if c in (0x130, 0x131):
            continue
        if icu:   # simple (single-rune) mappings and simple case folding
            maps = [icu.tolower(c), icu.toupper(c), icu.totitle(c), icu.fold(c, 0)]
        else:
            ch = chr(c)
            maps = [ord(m) for m in (ch.lower(), ch.upper(), ch.casefold()) if len(m) == 1]
        for m in maps:
            if m != c and m not in (0x130, 0x131):
                union(c, m)
    classes = {}
    nodes = set(parent) | set(parent.values())
    for c in nodes:
        classes.setdefault(find(c), set()).add(c)
    orbit = []   # (rune, next rune of its orbit, cyclic ascending) like unicode.SimpleFold
    for cl in classes.values():
        if len(cl) < 2:
            continue
        s = sorted(cl)
        for k, c in enumerate(s):
            orbit.append((c, s[(k + 1) % len(s)]))
    orbit.sort()

    w = sys.stdout.write
    if "--c" in sys.argv:   # oracle/unicode_data.c: plain C, the oracle's own data (test infrastructure)
        w("/* unicode_data.c — GENERATED by tools/gen_unicode_tables.py --c; do not edit.\n")
        w(" * Test infrastructure: the oracle's Unicode data (Unicode %s categories, scripts and\n"
          " * simple case-folding orbits; the regex module's Script property for scripts ICU lacks). */\n"
          % version)
        w('#include "oracle.h"\n\n')
        for kind, d in (("cat", tables), ("sc", scripts)):
            for nm, rs in d.items():
                flat = ",".join("%d,%d" % r for r in rs)
                w("static const int u_%s_%s[] = {%s};\n" % (kind, nm, flat or "0,0"))
        w("const orc_utab orc_ucats[] = {\n")
        for nm, rs in tables.items():
            w('  {"%s", u_cat_%s, %d},\n' % (nm, nm, len(rs)))
        w("};\nconst int orc_ucats_n = %d;\n" % len(tables))
        w("const orc_utab orc_uscripts[] = {\n")
        for nm, rs in scripts.items():
            w('  {"%s", u_sc_%s, %d},\n' % (nm, nm, len(rs)))
        w("};\nconst int orc_uscripts_n = %d;\n" % len(scripts))
        w("const int orc_fold_next[] = {%s};\n" % ",".join("%d,%d" % o for o in orbit))
        w("const int orc_fold_n = %d;\n" % len(orbit))
        return
    w("// unicode_tables.cpp — GENERATED by tools/gen_unicode_tables.py; do not edit.\n")
    w("// General categories, scripts and simple case mappings: Unicode %s (%s); scripts ICU does\n"
      % (version, "ICU" if icu else "Python unicodedata"))
    w("// not know: the regex module's Script property; simple case-folding orbits.\n")
    w("// Go 1.25 (the reference's regexp) uses Unicode 15.0.0: later code points are parity unpinned.\n")
    w('#include "unicode_tables.hpp"\n\nnamespace ose {\nnamespace {\n')
    names = []
    for kind, d in (("cat", tables), ("sc", scripts)):
        for nm, rs in d.items():
            ident = "k_%s_%s" % (kind, nm)
            flat = ",".join("0x%X,0x%X" % r for r in rs)
            w("const uint32_t %s[] = {%s};\n" % (ident, flat or "0,0"))
            names.append((kind, nm, ident, len(rs)))
    w("}  // namespace\n\n")
    w("const UniTable kUniCategories[] = {\n")
    for kind, nm, ident, n in names:
        if kind == "cat":
            w('    {"%s", %s, %d},\n' % (nm, ident, n))
    w("};\nconst uint32_t kUniCategoriesN = %d;\n" % sum(1 for x in names if x[0] == "cat"))
    w("const UniTable kUniScripts[] = {\n")
    for kind, nm, ident, n in names:
        if kind == "sc":
            w('    {"%s", %s, %d},\n' % (nm, ident, n))
    w("};\nconst uint32_t kUniScriptsN = %d;\n" % sum(1 for x in names if x[0] == "sc"))
    w("const uint32_t kFoldOrbit[] = {%s};\n" % ",".join("0x%X,0x%X" % o for o in orbit))
    w("const uint32_t kFoldOrbitN = %d;\n" % len(orbit))
    w("}  // namespace ose\n")


if __name__ == "__main__":
    main()

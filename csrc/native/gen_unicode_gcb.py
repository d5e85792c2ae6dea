"""Generate csrc/native/unicode_gcb.h: Grapheme_Cluster_Break ranges (UAX #29) for the
SentencePiece ``Precompiled`` normalizer (spm_norm.cpp), which -- like HF tokenizers -- maps
whole extended grapheme clusters.  Derived from Python's unicodedata (general categories) plus
the small property lists UAX #29 names that unicodedata does not expose (Other_Grapheme_Extend,
Prepend, Hangul syllable types, an Extended_Pictographic approximation).

    python csrc/native/gen_unicode_gcb.py   (writes the header; committed, so builds need no step)
"""
from __future__ import annotations

import os
import unicodedata

OTHER, CR, LF, CONTROL, EXTEND, ZWJ, RI, PREPEND, SPACING, L, V, T, LV, LVT, PICT = range(15)
NAMES = ["Other", "CR", "LF", "Control", "Extend", "ZWJ", "RI", "Prepend", "SpacingMark", "L", "V",
         "T", "LV", "LVT", "ExtPict"]

OTHER_GRAPHEME_EXTEND = [(0x09BE, 0x09BE), (0x09D7, 0x09D7), (0x0B3E, 0x0B3E), (0x0B57, 0x0B57),
                         (0x0BBE, 0x0BBE), (0x0BD7, 0x0BD7), (0x0CC2, 0x0CC2), (0x0CD5, 0x0CD6),
                         (0x0D3E, 0x0D3E), (0x0D57, 0x0D57), (0x0DCF, 0x0DCF), (0x0DDF, 0x0DDF),
                         (0x1B35, 0x1B35), (0x200C, 0x200C), (0x302E, 0x302F), (0xFF9E, 0xFF9F),
                         (0x1133E, 0x1133E), (0x11357, 0x11357), (0x114B0, 0x114B0),
                         (0x114BD, 0x114BD), (0x115AF, 0x115AF), (0x11930, 0x11930),
                         (0x1D165, 0x1D165), (0x1D16E, 0x1D172), (0xE0020, 0xE007F),
                         (0x1F3FB, 0x1F3FF)]   # (+ Emoji_Modifier, Extend since Unicode 11)
PREPEND_R = [(0x0600, 0x0605), (0x06DD, 0x06DD), (0x070F, 0x070F), (0x0890, 0x0891),
             (0x08E2, 0x08E2), (0x0D4E, 0x0D4E), (0x110BD, 0x110BD), (0x110CD, 0x110CD),
             (0x111C2, 0x111C3), (0x1193F, 0x1193F), (0x11941, 0x11941), (0x11A3A, 0x11A3A),
             (0x11A84, 0x11A89), (0x11D46, 0x11D46)]
NOT_SPACING = [(0x102B, 0x102C), (0x1038, 0x1038), (0x1062, 0x1064), (0x1067, 0x106D),
               (0x1083, 0x1083), (0x1087, 0x108C), (0x108F, 0x108F), (0x109A, 0x109C),
               (0x1A61, 0x1A61), (0x1A63, 0x1A64), (0xAA7B, 0xAA7B), (0xAA7D, 0xAA7D),
               (0x11720, 0x11721)]
PICT_R = [(0x00A9, 0x00A9), (0x00AE, 0x00AE), (0x203C, 0x203C), (0x2049, 0x2049),
          (0x2122, 0x2122), (0x2139, 0x2139), (0x2194, 0x2199), (0x21A9, 0x21AA),
          (0x231A, 0x231B), (0x2328, 0x2328), (0x2388, 0x2388), (0x23CF, 0x23CF),
          (0x23E9, 0x23F3), (0x23F8, 0x23FA), (0x24C2, 0x24C2), (0x25AA, 0x25AB),
          (0x25B6, 0x25B6), (0x25C0, 0x25C0), (0x25FB, 0x25FE), (0x2600, 0x2605),
          (0x2607, 0x2612), (0x2614, 0x2685), (0x2690, 0x2705), (0x2708, 0x2712),
          (0x2714, 0x2714), (0x2716, 0x2716), (0x271D, 0x271D), (0x2721, 0x2721),
          (0x2728, 0x2728), (0x2733, 0x2734), (0x2744, 0x2744), (0x2747, 0x2747),
          (0x274C, 0x274C), (0x274E, 0x274E), (0x2753, 0x2755), (0x2757, 0x2757),
          (0x2763, 0x2767), (0x2795, 0x2797), (0x27A1, 0x27A1), (0x27B0, 0x27B0),
          (0x27BF, 0x27BF), (0x2934, 0x2935), (0x2B05, 0x2B07), (0x2B1B, 0x2B1C),
          (0x2B50, 0x2B50), (0x2B55, 0x2B55), (0x3030, 0x3030), (0x303D, 0x303D),
          (0x3297, 0x3297), (0x3299, 0x3299), (0x1F000, 0x1F0FF), (0x1F10D, 0x1F10F),
          (0x1F12F, 0x1F12F), (0x1F16C, 0x1F171), (0x1F17E, 0x1F17F), (0x1F18E, 0x1F18E),
          (0x1F191, 0x1F19A), (0x1F1AD, 0x1F1E5), (0x1F201, 0x1F20F), (0x1F21A, 0x1F21A),
          (0x1F22F, 0x1F22F), (0x1F232, 0x1F23A), (0x1F23C, 0x1F23F), (0x1F249, 0x1F3FA),
          (0x1F400, 0x1F53D), (0x1F546, 0x1F64F), (0x1F680, 0x1F6FF), (0x1F774, 0x1F77F),
          (0x1F7D5, 0x1F7FF), (0x1F80C, 0x1F80F), (0x1F848, 0x1F84F), (0x1F85A, 0x1F85F),
          (0x1F888, 0x1F88F), (0x1F8AE, 0x1F8FF), (0x1F90C, 0x1F93A), (0x1F93C, 0x1F945),
          (0x1F947, 0x1FAFF), (0x1FC00, 0x1FFFD)]


def _in(cp, ranges):
    return any(a <= cp <= b for a, b in ranges)


def gcb(cp: int) -> int:
    if cp == 0x0D:
        return CR
    if cp == 0x0A:
        return LF
    if cp == 0x200D:
        return ZWJ
    if 0x1F1E6 <= cp <= 0x1F1FF:
        return RI
    if 0x1100 <= cp <= 0x115F or 0xA960 <= cp <= 0xA97C:
        return L
    if 0x1160 <= cp <= 0x11A7 or 0xD7B0 <= cp <= 0xD7C6:
        return V
    if 0x11A8 <= cp <= 0x11FF or 0xD7CB <= cp <= 0xD7FB:
        return T
    if 0xAC00 <= cp <= 0xD7A3:
        return LV if (cp - 0xAC00) % 28 == 0 else LVT
    if _in(cp, PREPEND_R):
        return PREPEND
    cat = unicodedata.category(chr(cp))
    if cat in ("Mn", "Me") or _in(cp, OTHER_GRAPHEME_EXTEND):
        return EXTEND
    if cat in ("Cc", "Zl", "Zp") or (cat == "Cf" and cp not in (0x200C, 0x200D)):
        return CONTROL
    if (cat == "Mc" and not _in(cp, NOT_SPACING)) or cp in (0x0E33, 0x0EB3):
        return SPACING
    if _in(cp, PICT_R):
        return PICT
    return OTHER


def main() -> None:
    ranges = []
    cur, start = None, 0
    for cp in range(0x110000):
        c = gcb(cp)
        if c != cur:
            if cur not in (None, OTHER):
                ranges.append((start, cp - 1, cur))
            cur, start = c, cp
    if cur != OTHER:
        ranges.append((start, 0x10FFFF, cur))
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "unicode_gcb.h")
    with open(out, "w") as f:
        f.write("// Generated by csrc/native/gen_unicode_gcb.py from Python's unicodedata "
                f"(Unicode {unicodedata.unidata_version}); do not edit.\n")
        f.write("// Grapheme_Cluster_Break ranges (lo, hi, class); every other code point is Other.\n")
        f.write("#pragma once\n#include <cstdint>\nnamespace symbn {\n")
        f.write("enum Gcb : uint8_t { " + ", ".join(f"kGcb{n} = {i}" for i, n in enumerate(NAMES))
                + " };\n")
        f.write("struct GcbRange { uint32_t lo, hi; uint8_t cls; };\n")
        f.write(f"static const GcbRange kGcbRanges[{len(ranges)}] = {{\n")
        for a, b, c in ranges:
            f.write(f"    {{0x{a:X}, 0x{b:X}, {c}}},\n")
        f.write("};\n}  // namespace symbn\n")
    print(f"{out}: {len(ranges)} ranges")


if __name__ == "__main__":
    main()

"""Extract the reference's printf format strings, in source order, as data.

The IPv4 / IPv6 parsers, show_frame_hdr and the SLL head cannot be compiled
here (proto_ipv4.c / proto_ipv6.c include geoip.h -> config.h, dissector.h
and dissector_sll.c include ring.h -> config.h, which only `configure`
generates).  Their *line layout* is pinned instead by reading
their `tprintf` calls out of the source text: each call's format string
(adjacent string literals and the colors.h colorize macros concatenated, C
escapes decoded) and those of its arguments that are literal text (a string
literal, a colorize expression, or a `cond ? lit : lit` choice), with the
line each call starts on.  tests/test_layout_pin.py checks that the oracle's
and the product formatter's text for these layers is exactly a sequence of
these strings along each control-flow path, with only the conversions
filled in.

Run in the build container (reads /root/reference as text; nothing is
compiled or executed from it):
    python tests/ref_formats.py            -> tests/golden/ref_formats.json
The committed JSON is a fixture of strings; no source file is copied.
"""
import json
import os
import re
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "golden", "ref_formats.json")

# (file, first line, last line, function) - the printers whose sources need config.h
RANGES = [
    ("proto_ipv4.c", 34, 178, "ipv4"),
    ("proto_ipv4.c", 180, 204, "ipv4_less"),
    ("proto_ipv6.c", 22, 95, "ipv6"),
    ("proto_ipv6.c", 97, 113, "ipv6_less"),
    ("dissector.h", 53, 108, "__show_frame_hdr"),
    ("dissector_sll.c", 39, 67, "sll_print_full"),
    ("dissector_sll.c", 69, 82, "sll_print_less"),
]


def color_macros():
    """colors.h's __name -> "digits" defines and the three colorize macros."""
    with open(os.path.join(REF, "colors.h")) as f:
        text = f.read()
    return dict(re.findall(r'#define\s+(__\w+)\s+"(\d+)"', text))


def decode_c(lit):
    """A C string literal body -> str (the escapes these files use)."""
    out, i = [], 0
    while i < len(lit):
        c = lit[i]
        if c != "\\":
            out.append(c)
            i += 1
            continue
        n = lit[i + 1]
        if n in "01234567":
            m = re.match(r"[0-7]{1,3}", lit[i + 1:])
            out.append(chr(int(m.group(0), 8)))
            i += 1 + len(m.group(0))
        elif n == "x":
            m = re.match(r"[0-9a-fA-F]+", lit[i + 2:])
            out.append(chr(int(m.group(0), 16)))
            i += 2 + len(m.group(0))
        else:
            out.append({"n": "\n", "t": "\t", "\\": "\\", '"': '"', "'": "'", "r": "\r"}[n])
            i += 2
    return "".join(out)


def literal_expr(expr, colors):
    """The text of a literal-only expression (string literals and colorize
    macros side by side), or None."""
    pos, parts = 0, []
    tok = re.compile(r'\s*(?:"((?:[^"\\]|\\.)*)"|colorize_start_full\((\w+),\s*(\w+)\)|'
                     r'colorize_start\((\w+)\)|colorize_end\(\))', re.S)
    expr = expr.strip()
    if not expr:
        return None
    while pos < len(expr):
        m = tok.match(expr, pos)
        if not m:
            return None
        if m.group(1) is not None:
            parts.append(decode_c(m.group(1)))
        elif m.group(2):
            parts.append("\033[" + colors["__" + m.group(2)] + ";" + colors["__on_" + m.group(3)] + "m")
        elif m.group(4):
            parts.append("\033[" + colors["__" + m.group(4)] + "m")
        else:
            parts.append("\033[" + colors["__reset"] + "m")
        pos = m.end()
        while pos < len(expr) and expr[pos].isspace():
            pos += 1
    return "".join(parts)


def split_args(s):
    """Top-level comma split of a call's argument text."""
    args, depth, cur, i = [], 0, [], 0
    while i < len(s):
        c = s[i]
        if c == '"':
            j = i + 1
            while s[j] != '"':
                j += 2 if s[j] == "\\" else 1
            cur.append(s[i:j + 1])
            i = j + 1
            continue
        if c in "([{":
            depth += 1
        elif c in ")]}":
            depth -= 1
        if c == "," and depth == 0:
            args.append("".join(cur))
            cur = []
        else:
            cur.append(c)
        i += 1
    args.append("".join(cur))
    return args


def arg_literal(a, colors):
    """A literal argument: its text, or for `cond ? lit : lit` the two
    choices [if-true, if-false]; None for a computed argument."""
    a = a.strip()
    lit = literal_expr(a, colors)
    if lit is not None:
        return lit
    # one level of ?: between literal expressions (string-aware split)
    depth, q = 0, None
    i = 0
    while i < len(a):
        c = a[i]
        if c == '"':
            j = i + 1
            while a[j] != '"':
                j += 2 if a[j] == "\\" else 1
            i = j + 1
            continue
        if c in "([":
            depth += 1
        elif c in ")]":
            depth -= 1
        elif c == "?" and depth == 0 and q is None:
            q = i
        elif c == ":" and depth == 0 and q is not None:
            t, f = literal_expr(a[q + 1:i], colors), literal_expr(a[i + 1:], colors)
            if t is not None and f is not None:
                return [t, f]
            return None
        i += 1
    return None


def extract(fname, lo, hi, func, colors):
    with open(os.path.join(REF, fname)) as f:
        lines = f.read().split("\n")
    # offsets of line starts
    text = "\n".join(lines)
    starts = [0]
    for ln in lines:
        starts.append(starts[-1] + len(ln) + 1)
    out = []
    for m in re.finditer(r"\btprintf\(", text):
        line = next(k for k in range(len(starts) - 1) if starts[k] <= m.start() < starts[k + 1]) + 1
        if not (lo <= line <= hi):
            continue
        # the call's argument text up to the matching parenthesis
        i, depth = m.end(), 1
        while depth:
            c = text[i]
            if c == '"':
                j = i + 1
                while text[j] != '"':
                    j += 2 if text[j] == "\\" else 1
                i = j + 1
                continue
            depth += c == "("
            depth -= c == ")"
            i += 1
        args = split_args(text[m.end():i - 1])
        fmt = literal_expr(args[0], colors)
        assert fmt is not None, (fname, line, args[0])
        out.append({"file": fname, "line": line, "func": func, "fmt": fmt,
                    "args": [arg_literal(a, colors) for a in args[1:]]})
    return out


# the string tables these printers print through: (file, first line, last
# line, name, pattern of one entry)
TABLES = [
    # packet_types[] (dissector.h:31-39): [PACKET_X] = "<"
    ("dissector.h", 31, 39, "packet_types", r"\[(PACKET_\w+)\]\s*=\s*\"((?:[^\"\\]|\\.)*)\""),
    # __show_ts_source's results (dissector.h:41-51), in test order
    ("dissector.h", 41, 51, "ts_source", r"()return\s+\"((?:[^\"\\]|\\.)*)\""),
    # pkt_type2str's results (dissector_sll.c:17-37): case PACKET_X: return "..."
    ("dissector_sll.c", 17, 37, "pkt_type2str", r"(?:case\s+(PACKET_\w+):\s*)?return\s+\"((?:[^\"\\]|\\.)*)\""),
]


def extract_table(fname, lo, hi, pat):
    with open(os.path.join(REF, fname)) as f:
        text = "\n".join(f.read().split("\n")[lo - 1:hi])
    return [[k or None, decode_c(v)] for k, v in re.findall(pat, text)]


def extract_all():
    colors = color_macros()
    calls = []
    for fname, lo, hi, func in RANGES:
        calls.extend(extract(fname, lo, hi, func, colors))
    tables = {name: extract_table(fname, lo, hi, pat) for fname, lo, hi, name, pat in TABLES}
    return {"calls": calls, "tables": tables}


def main():
    if not os.path.isdir(REF):
        sys.exit("needs /root/reference (build container only)")
    res = extract_all()
    with open(OUT, "w") as f:
        json.dump(res, f, indent=1, ensure_ascii=True)
        f.write("\n")
    print(f"{len(res['calls'])} tprintf calls, tables {sorted(res['tables'])} -> {os.path.relpath(OUT)}")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Remove retired diagnostic macros from a source file, keeping the code they left out (a small
unifdef: every listed macro is taken as undefined; directives that name only listed macros are
resolved, the others are kept as they are).

    python3 tools/strip_ifdefs.py FILE MACRO...
"""
import re
import sys


def cond_value(expr: str, gone: set):
    """True/False when expr only involves macros in `gone` (all undefined), else None."""
    names = set(re.findall(r"defined\s*\(\s*(\w+)\s*\)|defined\s+(\w+)", expr))
    names = {a or b for a, b in names}
    bare = set(re.findall(r"\b(TPZ_\w+)\b", expr)) - names
    if not names or (names | bare) - gone:
        return None
    py = re.sub(r"defined\s*\(\s*\w+\s*\)|defined\s+\w+", "False", expr)
    py = py.replace("&&", " and ").replace("||", " or ").replace("!", " not ")
    return bool(eval(py))


def strip(lines, gone):
    out = []
    # stack entries: (mode, taken) ; mode "keep" = directive kept verbatim, "res" = resolved
    stack = []
    active = lambda: all(e[0] == "keep" or e[1] == "on" for e in stack)  # noqa: E731
    for ln in lines:
        s = ln.strip()
        m = re.match(r"#\s*(ifdef|ifndef|if|elif|else|endif)\b(.*)", s)
        if not m:
            if active():
                out.append(ln)
            continue
        d, rest = m.group(1), m.group(2).split("//")[0].strip()
        if d in ("ifdef", "ifndef", "if"):
            expr = rest if d == "if" else ("defined(%s)" % rest if d == "ifdef" else "!defined(%s)" % rest)
            v = cond_value(expr, gone)
            if v is None:
                stack.append(["keep", None])
                if active():
                    out.append(ln)
            else:
                stack.append(["res", "on" if v else "off", v])
        elif d == "elif":
            top = stack[-1]
            if top[0] == "keep":
                if active():
                    out.append(ln)
            else:
                done = top[2]
                v = cond_value(rest, gone)
                if v is None:
                    raise SystemExit("mixed #elif after a resolved #if: " + ln)
                top[1] = "on" if (not done and v) else "off"
                top[2] = done or v
        elif d == "else":
            top = stack[-1]
            if top[0] == "keep":
                if active():
                    out.append(ln)
            else:
                top[1] = "off" if top[2] else "on"
                top[2] = True
        else:  # endif
            top = stack.pop()
            if top[0] == "keep" and active():
                out.append(ln)
    assert not stack
    return out


def main():
    path, gone = sys.argv[1], set(sys.argv[2:])
    lines = open(path).read().split("\n")
    open(path, "w").write("\n".join(strip(lines, gone)))


if __name__ == "__main__":
    main()

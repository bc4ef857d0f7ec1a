"""TEST INFRASTRUCTURE ONLY (never imported by the product path): a pure-Python
restatement of the reference's flat-netlist MNA front end, the checker for
gg_host_read_netlist.

  node rows     parser(), NodeList::findorPushNode   src/parser.cpp:69-272,
                src/element.cpp:95-130 (first appearance; "0"/"gnd" ground)
  G             stampG()   src/parser.cpp:1904-2099
  C             stampC()   src/parser.cpp:2100-2268
  B, sources    stampB()   src/parser.cpp:2269-2886
  suffixes      StrToNum() src/parser.cpp:30-67
  duplicates    matrix::pushEntry sums in push order, src/matrix.cpp:91-130

Parity unpinned against the reference itself: it ships no netlist fixtures and
its parser is not buildable here; this pins the C++ parser to
the restated rules on synthetic netlists."""
import math
import os
import re

SRC_DC, SRC_PULSE, SRC_PWL = 0, 1, 2


def str_to_num(s):
    m = re.match(r"\s*[-+]?(\d+\.?\d*|\.\d+)([eE][-+]?\d+)?", s)
    if not m:
        return 0.0
    v = float(m.group(0))
    rest = s[m.end():]
    c = rest[:1]
    if c in ("T", "t"):
        return v * math.pow(10.0, 12)
    if c in ("G", "g"):
        return v * math.pow(10.0, 9)
    if c in ("K", "k"):
        return v * math.pow(10.0, 3)
    if c in ("M", "m"):
        return v * math.pow(10.0, 6) if rest[1:2] in ("E", "e") else v * math.pow(10.0, -3)
    if c in ("U", "u"):
        return v * math.pow(10.0, -6)
    if c in ("n", "N"):
        return v * math.pow(10.0, -9)
    if c in ("p", "P"):
        return v * math.pow(10.0, -12)
    if c in ("f", "F"):
        return v * math.pow(10.0, -15)
    return v


def _lines(path, depth=0):
    out = []
    d = os.path.dirname(path)
    with open(path) as f:
        for l in f.read().split("\n"):
            l = l.rstrip("\r")
            if depth == 0 and l.startswith(".in"):
                t = l.split()
                if len(t) >= 2:
                    out += _lines(os.path.join(d, t[1].replace('"', "")), 1)
                    continue
            out.append(l)
    return out


def _check_element(t, l):
    # both passes: an element line needs a name, two nodes and a value
    if len(t) < 4:
        raise ValueError(f"netlist: element line needs a name, two nodes and a value: {l!r}")


def _pulse_args(l, kw):
    # the numbers between the '(' after the PULSE keyword and the next ')',
    # blank- and/or comma-separated (the reference's spelling reads the same
    # values as its sscanf, src/parser.cpp:2655-2686); fewer than 7: None
    a = l.find("(", kw)
    if a < 0:
        return None
    b = l.find(")", a)
    body = l[a + 1:(b if b >= 0 else len(l))].replace(",", " ").split()
    return [str_to_num(x) for x in body[:7]] if len(body) >= 7 else None


def read_netlist(path):
    """dict: n, n_nodes, n_l, n_v, n_i, tstep, tstop, G, C, B as
    {(i, j): value} accumulated in push order, sources [(kind, [params])],
    ports [row or -1]"""
    lines = _lines(path)
    rows, nn = {}, [0]

    def node(nm):
        if nm not in rows:
            if nm in ("0", "gnd"):
                rows[nm] = -1
            else:
                rows[nm] = nn[0]
                nn[0] += 1
        return rows[nm]

    nl = nv = ni = 0
    tstep = tstop = 0.0
    ports = []
    for l in lines:
        if not l:
            continue
        c = l[0].upper()
        if c in "RCLVI":
            t = l.split()
            _check_element(t, l)
            nl += c == "L"
            nv += c == "V"
            ni += c == "I"
            node(t[1])
            node(t[2])
        elif c == "." and len(l) > 1:
            if l[1] == "t":
                t = l.split()
                if len(t) >= 3:
                    tstep, tstop = str_to_num(t[1]), str_to_num(t[2])
            elif l[1:3] == "pr":
                ports += re.findall(r"\(([^)]*)\)", l)
    nnodes = nn[0]
    G, C, B = {}, {}, {}

    def push(M, i, j, v):
        M[(i, j)] = M[(i, j)] + v if (i, j) in M else v

    src = [None] * (nv + ni)
    il, iv, ii = 0, -1, -1
    last = None
    for l in lines:
        if not l:
            continue
        c = l[0].upper()
        t = l.split()
        if c == "+":
            p = l[2:].split()
            if last is not None and len(p) >= 2:
                tm, v = str_to_num(p[0]), str_to_num(p[1])
                if not last[1] and tm != 0.0:
                    last[1] += [0.0, v]
                last[1] += [tm, v]
            continue
        if c not in "RCLVI":
            continue
        _check_element(t, l)
        iv += c == "V"
        ii += c == "I"
        n1, n2 = rows[t[1]], rows[t[2]]
        if c in "RC":
            v = 1.0 / str_to_num(t[3]) if c == "R" else str_to_num(t[3])
            M = G if c == "R" else C
            if n1 >= 0:
                push(M, n1, n1, v)
            if n2 >= 0:
                push(M, n2, n2, v)
            if n1 >= 0 and n2 >= 0:
                push(M, n1, n2, -v)
                push(M, n2, n1, -v)
        elif c == "L":
            k = nnodes + il
            il += 1
            if n1 >= 0:
                push(G, k, n1, -1.0)
                push(G, n1, k, 1.0)
            if n2 >= 0:
                push(G, k, n2, 1.0)
                push(G, n2, k, -1.0)
            push(C, k, k, str_to_num(t[3]))
        else:
            j = iv if c == "V" else nv + ii
            if c == "V":
                k = nnodes + nl + iv
                if n1 >= 0:
                    push(G, n1, k, 1.0)
                    push(G, k, n1, -1.0)
                if n2 >= 0:
                    push(G, n2, k, -1.0)
                    push(G, k, n2, 1.0)
                push(B, k, j, -1.0)
            else:
                if n1 >= 0:
                    push(B, n1, j, -1.0)
                if n2 >= 0:
                    push(B, n2, j, 1.0)
            w = t[3]
            s = [SRC_DC, []]
            if w[:2].upper() == "PW":
                s[0] = SRC_PWL
                a = l.find("(")
                b = l.find(")", a)
                body = l[a + 1:(b if b >= 0 else len(l))].split() if a >= 0 else []
                for q in range(0, len(body) - 1, 2):
                    tm, v = str_to_num(body[q]), str_to_num(body[q + 1])
                    if not s[1] and tm != 0.0:
                        s[1] += [0.0, v]
                    s[1] += [tm, v]
            elif len(t) >= 5 and t[4][:2].upper() == "PU":
                q = _pulse_args(l, l.find(t[4]))
                s = [SRC_PULSE, q] if q is not None else [SRC_DC, [0.0]]
            else:
                s = [SRC_DC, [str_to_num(w)]]
            src[j] = s
            last = s
    return dict(n=nnodes + nl + nv, n_nodes=nnodes, n_l=nl, n_v=nv, n_i=ni, tstep=tstep,
                tstop=tstop, G=G, C=C, B=B, sources=[(k, list(p)) for k, p in src],
                ports=[rows.get(p, -1) for p in ports])

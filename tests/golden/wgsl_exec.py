"""A small WGSL interpreter -- TEST INFRASTRUCTURE ONLY: used by
tests/golden/make_wgsl_golden.py (fixture generation from the reference's
shaders, in the build container) and by its own self-tests
(tests/test_wgsl_exec.py, inline snippets); never imported by the product.

It parses the subset of WGSL (naga 0.9 dialect) that the reference's compute
shaders use and executes a kernel invocation by invocation on the CPU, with
IEEE-754 binary32 arithmetic: every f32 operation is one numpy float32
round-to-nearest op in the order the expression is written (no FMA
contraction), u32/i32 wrap modulo 2^32. The WGSL builtins whose precision the
WGSL spec leaves to the driver take the op forms the oracle fixes
(oracle/rt_oracle.c header): dot = (x*x' + y*y') + z*z', length = sqrt(dot),
normalize = v / length (three divides), sqrt correctly rounded, pow(x, 5.0) =
((x*x)*(x*x))*x, tan/cos/sin = the double-precision function rounded to f32,
min/max as C fminf/fmaxf, M * v = ((c0*x + c1*y) + c2*z) + c3*w.

Buffers are decoded from bytes with the WGSL host-shareable layout rules
(vec3 align 16 size 12, runtime-array stride = roundUp(align, size)), so the
host records are read exactly as the reference's shaders would read them.
"""
from __future__ import annotations

import math
import re
import struct as _struct

import numpy as np

F32, U32, I32 = np.float32, np.uint32, np.int32
M32 = 0xFFFFFFFF

_TOK = re.compile(r"""
 (?P<ws>\s+|//[^\n]*)
|(?P<num>0[xX][0-9a-fA-F]+[ui]?|(?:\d+\.\d*|\.\d+|\d+)(?:[eE][+-]?\d+)?[fuih]?)
|(?P<id>[A-Za-z_][A-Za-z0-9_]*)
|(?P<attr>@[A-Za-z_]+)
|(?P<op><<=|>>=|<<|>>|<=|>=|==|!=|&&|\|\||\+=|-=|\*=|/=|%=|&=|\|=|\^=|->|[-+*/%<>=!&|^~(){}\[\],;:.])
""", re.X)

GENERIC = {"vec2", "vec3", "vec4", "mat4x4", "mat3x3", "array", "atomic", "ptr",
           "texture_storage_2d"}


def tokenize(src):
    out, pos = [], 0
    while pos < len(src):
        m = _TOK.match(src, pos)
        if not m:
            raise SyntaxError(f"bad char {src[pos]!r} at {pos}")
        pos = m.end()
        if m.lastgroup != "ws":
            out.append((m.lastgroup, m.group()))
    out.append(("eof", ""))
    return out


def parse_number(s):
    low = s.lower()
    if low.startswith("0x"):
        if low.endswith("u"):
            return U32(int(low[2:-1], 16))
        if low.endswith("i"):
            return I32(int(low[2:-1], 16))
        return int(low[2:], 16)
    if low.endswith("f"):
        return F32(float(low[:-1]))
    if low.endswith("u"):
        return U32(int(low[:-1]))
    if low.endswith("i"):
        return I32(int(low[:-1]))
    if any(c in low for c in ".e"):
        return float(low)  # abstract float
    return int(low)  # abstract int


# ---------------------------------------------------------------- values
class Vec(tuple):
    pass


class Mat:
    __slots__ = ("cols",)

    def __init__(self, cols):
        self.cols = cols


class Struct:
    __slots__ = ("name", "f")

    def __init__(self, name, f):
        self.name, self.f = name, f

    def copy(self):
        return Struct(self.name, {k: cp(v) for k, v in self.f.items()})


def cp(v):
    return v.copy() if isinstance(v, Struct) else v


def concrete(v, k):
    """Convert an abstract (Python) literal to the scalar kind k."""
    if k == "f":
        return F32(v)
    if k == "u":
        return U32(int(v) & M32)
    if k == "i":
        return I32(((int(v) + 2**31) & M32) - 2**31)
    return v


def kind(v):
    t = type(v)
    if t is F32:
        return "f"
    if t is U32:
        return "u"
    if t is I32:
        return "i"
    if t is bool or t is np.bool_:
        return "b"
    if t is float:
        return "af"
    if t is int:
        return "ai"
    raise TypeError(f"not a scalar: {v!r}")


def default_kind(v):
    k = kind(v)
    return {"af": "f", "ai": "i"}.get(k, k)


def wrap(k, x):
    if k == "u":
        return U32(x & M32)
    if k == "i":
        return I32(((x + 2**31) & M32) - 2**31)
    return x


def sbin(op, a, b):
    ka, kb = kind(a), kind(b)
    if ka[0] == "a" and kb[0] != "a":
        a, ka = concrete(a, kb), kb
    elif kb[0] == "a" and ka[0] != "a":
        b, kb = concrete(b, ka), ka
    if op in ("==", "!=", "<", ">", "<=", ">="):
        return {"==": a == b, "!=": a != b, "<": a < b, ">": a > b,
                "<=": a <= b, ">=": a >= b}[op].__bool__()
    k = ka
    if k == "f":
        if op == "+":
            return a + b
        if op == "-":
            return a - b
        if op == "*":
            return a * b
        if op == "/":
            return a / b
        if op == "%":
            return F32(np.fmod(a, b))
    elif k in ("u", "i"):
        x, y = int(a), int(b)
        if op == "+":
            return wrap(k, x + y)
        if op == "-":
            return wrap(k, x - y)
        if op == "*":
            return wrap(k, x * y)
        if op == "/":
            q = abs(x) // abs(y)
            return wrap(k, q if (x >= 0) == (y >= 0) else -q)
        if op == "%":
            r = abs(x) % abs(y)
            return wrap(k, r if x >= 0 else -r)
        if op == "<<":
            return wrap(k, x << (y & 31))
        if op == ">>":
            return wrap(k, x >> (y & 31))
        if op == "&":
            return wrap(k, x & y)
        if op == "|":
            return wrap(k, x | y)
        if op == "^":
            return wrap(k, x ^ y)
    elif k in ("af", "ai"):
        return {"+": a + b, "-": a - b, "*": a * b}.get(op) if op in "+-*" else (
            a / b if k == "af" else int(a / b))
    elif k == "b":
        if op == "&":
            return a and b
        if op == "|":
            return a or b
    raise TypeError(f"{op} on {ka},{kb}")


def vbin(op, a, b):
    va, vb = isinstance(a, Vec), isinstance(b, Vec)
    if isinstance(a, Mat):
        assert op == "*" and vb and len(b) == 4
        acc = None
        for c, s in zip(a.cols, b):  # ((c0*x + c1*y) + c2*z) + c3*w
            t = vbin("*", c, s)
            acc = t if acc is None else vbin("+", acc, t)
        return acc
    if va and vb:
        r = [sbin(op, x, y) for x, y in zip(a, b)]
    elif va:
        r = [sbin(op, x, b) for x in a]
    elif vb:
        r = [sbin(op, a, y) for y in b]
    else:
        return sbin(op, a, b)
    return r if op in ("==", "!=", "<", ">", "<=", ">=") else Vec(r)


def neg(v):
    if isinstance(v, Vec):
        return Vec(neg(x) for x in v)
    k = kind(v)
    if k == "f":
        return -v
    if k in ("u", "i"):
        return wrap(k, -int(v))
    return -v


# ------------------------------------------------------------------ parser
class Parser:
    def __init__(self, src):
        self.t = tokenize(src)
        self.i = 0

    def peek(self, o=0):
        return self.t[self.i + o]

    def next(self):
        tok = self.t[self.i]
        self.i += 1
        return tok

    def accept(self, v):
        if self.t[self.i][1] == v:
            self.i += 1
            return True
        return False

    def expect(self, v):
        tok = self.next()
        if tok[1] != v:
            raise SyntaxError(f"expected {v!r}, got {tok[1]!r} at token {self.i}")
        return tok

    def ident(self):
        tok = self.next()
        if tok[0] != "id":
            raise SyntaxError(f"expected identifier, got {tok[1]!r}")
        return tok[1]

    def attrs(self):
        while self.peek()[0] == "attr":
            self.next()
            if self.accept("("):
                depth = 1
                while depth:
                    v = self.next()[1]
                    depth += (v == "(") - (v == ")")

    def type_(self):
        name = self.ident()
        args = []
        if self.accept("<"):
            while True:
                args.append(self.type_())
                if self.accept(">"):
                    break
                self.expect(",")
        return (name, tuple(args))

    # module
    def module(self):
        m = {"consts": [], "structs": {}, "vars": {}, "fns": {}}
        while self.peek()[0] != "eof":
            self.attrs()
            tok = self.peek()[1]
            if tok == "struct":
                self.next()
                name = self.ident()
                self.expect("{")
                fields = []
                while not self.accept("}"):
                    self.attrs()
                    fname = self.ident()
                    self.expect(":")
                    fields.append((fname, self.type_()))
                    self.accept(",")
                self.accept(";")
                m["structs"][name] = fields
            elif tok in ("let", "const"):
                self.next()
                name = self.ident()
                ty = self.type_() if self.accept(":") else None
                self.expect("=")
                e = self.expr()
                self.expect(";")
                m["consts"].append((name, ty, e))
            elif tok == "var":
                self.next()
                space = []
                if self.accept("<"):
                    while not self.accept(">"):
                        space.append(self.ident())
                        self.accept(",")
                name = self.ident()
                self.expect(":")
                ty = self.type_()
                self.expect(";")
                m["vars"][name] = (tuple(space), ty)
            elif tok == "fn":
                self.next()
                name = self.ident()
                self.expect("(")
                params = []
                while not self.accept(")"):
                    self.attrs()
                    pname = self.ident()
                    self.expect(":")
                    params.append((pname, self.type_()))
                    self.accept(",")
                ret = self.type_() if self.accept("->") else None
                m["fns"][name] = (params, ret, self.block())
            elif tok == ";":
                self.next()
            else:
                raise SyntaxError(f"unexpected {tok!r} at module scope")
        return m

    def block(self):
        self.expect("{")
        body = []
        while not self.accept("}"):
            s = self.stmt()
            if s is not None:
                body.append(s)
        return ("block", body)

    def simple_stmt(self):
        tok = self.peek()[1]
        if tok in ("var", "let", "const"):
            self.next()
            name = self.ident()
            ty = self.type_() if self.accept(":") else None
            e = self.expr() if self.accept("=") else None
            return ("decl", tok, name, ty, e)
        e = self.expr()
        op = self.peek()[1]
        if op in ("=", "+=", "-=", "*=", "/=", "%=", "&=", "|=", "^=", "<<=", ">>="):
            self.next()
            return ("assign", op, e, self.expr())
        return ("expr", e)

    def stmt(self):
        tok = self.peek()[1]
        if tok == ";":
            self.next()
            return None
        if tok == "{":
            return self.block()
        if tok == "if":
            self.next()
            cond = self.expr()
            then = self.block()
            els = None
            if self.accept("else"):
                els = self.stmt() if self.peek()[1] == "if" else self.block()
            return ("if", cond, then, els)
        if tok == "for":
            self.next()
            self.expect("(")
            init = None if self.peek()[1] == ";" else self.simple_stmt()
            self.expect(";")
            cond = None if self.peek()[1] == ";" else self.expr()
            self.expect(";")
            upd = None if self.peek()[1] == ")" else self.simple_stmt()
            self.expect(")")
            return ("for", init, cond, upd, self.block())
        if tok == "return":
            self.next()
            e = None if self.peek()[1] == ";" else self.expr()
            self.expect(";")
            return ("ret", e)
        if tok in ("break", "continue"):
            self.next()
            self.expect(";")
            return (tok,)
        s = self.simple_stmt()
        self.expect(";")
        return s

    PREC = [("||",), ("&&",), ("|",), ("^",), ("&",), ("==", "!="), ("<", ">", "<=", ">="),
            ("<<", ">>"), ("+", "-"), ("*", "/", "%")]

    def expr(self, level=0):
        if level == len(self.PREC):
            return self.unary()
        lhs = self.expr(level + 1)
        while self.peek()[1] in self.PREC[level]:
            op = self.next()[1]
            lhs = ("bin", op, lhs, self.expr(level + 1))
        return lhs

    def unary(self):
        tok = self.peek()[1]
        if tok in ("-", "!", "~"):
            self.next()
            return ("un", tok, self.unary())
        if tok == "&":
            self.next()
            return ("addr", self.unary())
        return self.postfix(self.primary())

    def primary(self):
        kind_, v = self.next()
        if kind_ == "num":
            return ("lit", parse_number(v))
        if v == "(":
            e = self.expr()
            self.expect(")")
            return e
        if kind_ == "id":
            if v in ("true", "false"):
                return ("lit", v == "true")
            targs = ()
            if v in GENERIC and self.peek()[1] == "<":
                self.i -= 1
                v, targs = self.type_()
            if self.peek()[1] == "(":
                self.next()
                args = []
                while not self.accept(")"):
                    args.append(self.expr())
                    self.accept(",")
                return ("call", v, targs, args)
            return ("id", v)
        raise SyntaxError(f"unexpected {v!r}")

    def postfix(self, e):
        while True:
            if self.accept("."):
                e = ("mem", e, self.ident())
            elif self.accept("["):
                idx = self.expr()
                self.expect("]")
                e = ("idx", e, idx)
            else:
                return e


# ------------------------------------------------------------ interpreter
_SIG_BREAK, _SIG_CONT = object(), object()
_SW = {"x": 0, "y": 1, "z": 2, "w": 3, "r": 0, "g": 1, "b": 2, "a": 3}


def _fmin(a, b):
    return b if a != a else (a if b != b else (a if a < b else b))


def _fmax(a, b):
    return b if a != a else (a if b != b else (a if a > b else b))


def _dot(a, b):
    r = a[0] * b[0]
    for x, y in zip(a[1:], b[1:]):
        r = r + x * y
    return r


def _length(v):
    return F32(np.sqrt(_dot(v, v))) if isinstance(v, Vec) else F32(abs(v))


def _normalize(v):
    l = _length(v)
    return Vec(x / l for x in v)


def _pow(x, y):
    if float(y) != 5.0:
        raise NotImplementedError("pow: only the exponent 5.0 appears in the reference")
    x2 = x * x
    return (x2 * x2) * x


def _map1(fn, v):
    return Vec(fn(x) for x in v) if isinstance(v, Vec) else fn(v)


class Shader:
    """One parsed WGSL module bound to host resources."""

    def __init__(self, src):
        self.m = Parser(src).module()
        self.structs = self.m["structs"]
        self.consts = {}
        for name, ty, e in self.m["consts"]:
            v = self.eval(e, [{}])
            self.consts[name] = self.convert(v, ty) if ty else concrete(v, default_kind(v))
        self.res = {}

    # ---- layout (WGSL host-shareable rules)
    def layout(self, ty):
        name, args = ty
        if name in ("f32", "u32", "i32", "atomic"):
            return 4, 4
        if name.startswith("vec"):
            n = int(name[3])
            return (8 if n == 2 else 16), 4 * n
        if name == "mat4x4":
            return 16, 64
        if name in self.structs:
            off, al = 0, 1
            for _, fty in self.structs[name]:
                a, s = self.layout(fty)
                off = -(-off // a) * a + s
                al = max(al, a)
            return al, -(-off // al) * al
        raise TypeError(f"no layout for {ty}")

    def decode(self, ty, buf, off=0):
        name, args = ty
        if name == "atomic":
            return self.decode(args[0], buf, off)
        if name == "f32":
            return F32(_struct.unpack_from("<f", buf, off)[0])
        if name == "u32":
            return U32(_struct.unpack_from("<I", buf, off)[0])
        if name == "i32":
            return I32(_struct.unpack_from("<i", buf, off)[0])
        if name.startswith("vec"):
            n = int(name[3])
            return Vec(self.decode(args[0], buf, off + 4 * i) for i in range(n))
        if name == "mat4x4":
            return Mat([self.decode(("vec4", args), buf, off + 16 * c) for c in range(4)])
        if name in self.structs:
            f, o = {}, 0
            for fname, fty in self.structs[name]:
                if fty[0] == "array":  # runtime-sized array: to the end of the buffer
                    a, s = self.layout(fty[1][0])
                    o = -(-o // a) * a
                    stride = -(-s // a) * a
                    cnt = (len(buf) - off - o) // stride
                    f[fname] = [self.decode(fty[1][0], buf, off + o + k * stride)
                                for k in range(cnt)]
                    continue
                a, s = self.layout(fty)
                o = -(-o // a) * a
                f[fname] = self.decode(fty, buf, off + o)
                o += s
            return Struct(name, f)
        raise TypeError(f"cannot decode {ty}")

    def var_type(self, name):
        return self.m["vars"][name][1]

    def bind(self, **res):
        self.res.update(res)

    # ---- conversion
    def convert(self, v, ty):
        name, args = ty
        if name == "f32":
            return F32(v) if kind(v) != "f" else v
        if name == "u32":
            return v if kind(v) == "u" else U32(int(v) & M32)
        if name == "i32":
            return v if kind(v) == "i" else concrete(int(v), "i")
        if name.startswith("vec"):
            return Vec(self.convert(x, args[0]) if args else x for x in v)
        if name == "atomic":
            return self.convert(v, args[0])
        return cp(v)

    def construct(self, name, targs, vals):
        if name in ("f32", "u32", "i32"):
            v = vals[0]
            if name == "f32":
                return F32(v)
            k = kind(v)
            if k in ("f", "af"):
                x = math.trunc(float(v))
            else:
                x = int(v)
            return concrete(x, name[0])
        if name.startswith("vec"):
            n = int(name[3])
            comps = []
            for v in vals:
                comps.extend(v if isinstance(v, Vec) else [v])
            if len(comps) == 1:
                comps = comps * n
            assert len(comps) == n, (name, len(comps))
            if targs:
                return Vec(self.convert(c, targs[0]) for c in comps)
            k = next((kind(c) for c in comps if kind(c)[0] != "a"), None)
            k = k or default_kind(comps[0])
            return Vec(concrete(c, k) if kind(c)[0] == "a" else c for c in comps)
        if name in self.structs:
            return Struct(name, {fn: self.convert(v, ft)
                                 for (fn, ft), v in zip(self.structs[name], vals)})
        raise NameError(name)

    # ---- references
    def lookup(self, name, env):
        for scope in reversed(env):
            if name in scope:
                return scope[name]
        if name in self.consts:
            return self.consts[name]
        return self.res[name]

    def ref(self, e, env):
        """(container, key) of an lvalue."""
        t = e[0]
        if t == "id":
            for scope in reversed(env):
                if e[1] in scope:
                    return scope, e[1]
            return self.res, e[1]
        if t == "mem":
            c, k = self.ref(e[1], env)
            base = c[k]
            if isinstance(base, Struct):
                return base.f, e[2]
            raise TypeError(f"cannot assign to component .{e[2]}")
        if t == "idx":
            c, k = self.ref(e[1], env)
            return c[k], int(self.eval(e[2], env))
        raise TypeError(f"not an lvalue: {e}")

    # ---- evaluation
    def eval(self, e, env):
        t = e[0]
        if t == "lit":
            return e[1]
        if t == "id":
            return self.lookup(e[1], env)
        if t == "bin":
            op = e[1]
            if op == "&&":
                return bool(self.eval(e[2], env)) and bool(self.eval(e[3], env))
            if op == "||":
                return bool(self.eval(e[2], env)) or bool(self.eval(e[3], env))
            return vbin(op, self.eval(e[2], env), self.eval(e[3], env))
        if t == "mem":
            base = self.eval(e[1], env)
            f = e[2]
            if isinstance(base, Struct):
                return base.f[f]
            if isinstance(base, Mat):
                return base.cols[_SW[f]]
            if len(f) == 1:
                return base[_SW[f]]
            return Vec(base[_SW[c]] for c in f)
        if t == "idx":
            base = self.eval(e[1], env)
            i = int(self.eval(e[2], env))
            if isinstance(base, Mat):
                return base.cols[i]
            return base[i]
        if t == "un":
            v = self.eval(e[2], env)
            if e[1] == "-":
                return neg(v)
            if e[1] == "!":
                return not v
            return wrap(kind(v), ~int(v))
        if t == "addr":
            return self.ref(e[1], env)
        if t == "call":
            return self.call(e, env)
        raise TypeError(t)

    def call(self, e, env):
        _, name, targs, args = e
        if name in self.m["fns"]:
            params, ret, body = self.m["fns"][name]
            scope = {p: self.convert(cp(self.eval(a, env)), pt)
                     for (p, pt), a in zip(params, args)}
            sig = self.exec(body, [scope])
            if isinstance(sig, tuple):
                v = sig[1]
                return self.convert(v, ret) if ret else v
            return None
        if name == "atomicAdd":
            c, k = self.eval(args[0], env)
            old = c[k]
            c[k] = vbin("+", old, self.eval(args[1], env))
            return old
        if name == "storageBarrier":
            return None
        if name == "textureStore":
            tex = self.eval(args[0], env)
            xy = self.eval(args[1], env)
            v = self.eval(args[2], env)
            tex[int(xy[1]), int(xy[0])] = [float(c) for c in v]
            return None
        vals = [self.eval(a, env) for a in args]
        if name == "dot":
            return _dot(*vals)
        if name == "length":
            return _length(vals[0])
        if name == "normalize":
            return _normalize(vals[0])
        if name == "sqrt":
            return _map1(lambda x: F32(np.sqrt(F32(x))), vals[0])
        if name == "abs":
            return _map1(lambda x: F32(abs(F32(x))) if kind(x) in ("f", "af") else abs(x), vals[0])
        if name == "floor":
            return _map1(lambda x: F32(np.floor(F32(x))), vals[0])
        if name in ("tan", "cos", "sin"):
            fn = getattr(math, name)
            return _map1(lambda x: F32(fn(float(F32(x)))), vals[0])
        if name == "pow":
            return _pow(F32(vals[0]), vals[1])
        if name in ("min", "max"):
            a, b = vals
            if kind(a)[0] == "a" and kind(b)[0] != "a":
                a = concrete(a, kind(b))
            if kind(b)[0] == "a" and kind(a)[0] != "a":
                b = concrete(b, kind(a))
            if kind(a) == "f":
                return (_fmin if name == "min" else _fmax)(a, b)
            return min(a, b) if name == "min" else max(a, b)
        return self.construct(name, targs, vals)

    def exec(self, s, env):
        t = s[0]
        if t == "block":
            env.append({})
            try:
                for st in s[1]:
                    sig = self.exec(st, env)
                    if sig is not None:
                        return sig
            finally:
                env.pop()
            return None
        if t == "decl":
            _, kw, name, ty, e = s
            v = self.eval(e, env) if e is not None else None
            if ty is not None:
                v = self.convert(v, ty)
            elif not isinstance(v, (Vec, Struct, Mat, tuple)):
                v = concrete(v, default_kind(v)) if kind(v)[0] == "a" else v
            env[-1][name] = cp(v)
            return None
        if t == "assign":
            _, op, lhs, rhs = s
            c, k = self.ref(lhs, env)
            v = self.eval(rhs, env)
            if op != "=":
                v = vbin(op[:-1], c[k], v)
            old = c[k]
            if not isinstance(v, (Vec, Struct, Mat)) and kind(v)[0] == "a":
                v = concrete(v, kind(old))
            c[k] = cp(v)
            return None
        if t == "expr":
            self.eval(s[1], env)
            return None
        if t == "if":
            if self.eval(s[1], env):
                return self.exec(s[2], env)
            if s[3] is not None:
                return self.exec(s[3], env)
            return None
        if t == "for":
            _, init, cond, upd, body = s
            env.append({})
            try:
                if init is not None:
                    self.exec(init, env)
                while cond is None or self.eval(cond, env):
                    sig = self.exec(body, env)
                    if sig is _SIG_BREAK:
                        break
                    if isinstance(sig, tuple):
                        return sig
                    if upd is not None:
                        self.exec(upd, env)
            finally:
                env.pop()
            return None
        if t == "ret":
            return ("ret", self.eval(s[1], env) if s[1] is not None else None)
        if t == "break":
            return _SIG_BREAK
        if t == "continue":
            return _SIG_CONT
        raise TypeError(t)

    def dispatch(self, entry, groups, workgroup_size):
        """Run `entry` for every invocation of a 1-D dispatch, in order."""
        params, _, body = self.m["fns"][entry]
        pname = params[0][0]
        with np.errstate(all="ignore"):
            for gid in range(groups * workgroup_size):
                self.exec(body, [{pname: Vec((U32(gid), U32(0), U32(0)))}])


"""CPU restatement of Cedar policy parsing + authorization — TEST INFRASTRUCTURE ONLY.

This module is the *oracle* for the MI355X evaluator. Only `tests/`, `__graft_entry__.smoke()`
and `bench.py`'s `cpu_baseline` leg may import it, and only as the checker. The product path
(`cedar-access-control-for-k8s_amd/`) never imports it.

What it restates
----------------
The reference webhook (pure Go) delegates all Cedar arithmetic to the third-party module
`github.com/cedar-policy/cedar-go v1.1.0` (reference `go.mod:10`, `go.sum:41-42`), which is not
vendored and cannot be fetched here (no network, no Go toolchain). This file restates the
published Cedar language semantics as cedar-go v1.1.0 implements them, anchored on the reference's
own call sites:

* `cedar.NewPolicySetFromBytes(filename, doc)` — memory store, IDs ``policy<i>``
  (`internal/server/store/memory.go:17-27`, pinned by `store_test.go:102-103`,
  `authorizer_test.go:504`).
* `cedar.NewPolicyListFromBytes` + ``<file>.policy<i>`` IDs (`store/directory.go:69-77`),
  ``<name><i>-<uid>`` (`store/crd.go:60`), ``<id>.<i>`` (`store/verified_permissions.go:95`).
* `(*cedar.PolicySet).IsAuthorized(entities, req)` (call site `store/store.go:31`): every policy is
  evaluated; erroring policies are skipped and reported; any satisfied forbid -> Deny with the
  forbids as reasons; else any satisfied permit -> Allow with the permits as reasons; else Deny
  with no reasons. Errors are always reported.
* `TieredPolicyStores.IsAuthorized` (`store/store.go:25-42`).

Pinning: see `tests/test_oracle_golden.py` — the oracle reproduces every decision and exact reason
string of the reference's `TestAuthorize` (13 cases, `authorizer_test.go:462-920`), the 3 tier
cases of `TestTieredIsAuthorized` (`store_test.go:21-188`), and parses the 13 converter golden
`.cedar` files (`internal/convert/testdata/`) plus both demo policy files.

Canonicalisation (parity unpinned upstream): cedar-go keeps policies in a Go map, so the order of
multiple reasons/errors is not defined by the reference. The oracle emits them in policy insertion
order. Error message texts are not pinned by any reference test; they are rendered in cedar-go's
style and compared only where both sides are ours.
"""
from __future__ import annotations

import ipaddress
import re
import json
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

# ----------------------------------------------------------------------------------------------
# Values
# ----------------------------------------------------------------------------------------------

LONG_MIN = -(1 << 63)
LONG_MAX = (1 << 63) - 1


class Long:
    """Cedar Long (int64). Wrapped so that ``Long(1) != True`` inside Python sets."""

    __slots__ = ("v",)

    def __init__(self, v: int):
        self.v = int(v)

    def __eq__(self, o):
        return isinstance(o, Long) and o.v == self.v

    def __hash__(self):
        return hash(("L", self.v))

    def __repr__(self):
        return f"Long({self.v})"


@dataclass(frozen=True)
class EntityUID:
    type: str
    id: str

    def __str__(self):
        return f"{self.type}::{go_quote(self.id)}"


class CSet:
    """Cedar Set: unordered, duplicate-free, structural equality."""

    __slots__ = ("items",)

    def __init__(self, items=()):
        self.items = frozenset(items)

    def __eq__(self, o):
        return isinstance(o, CSet) and o.items == self.items

    def __hash__(self):
        return hash(("S", self.items))

    def __iter__(self):
        return iter(self.items)

    def __len__(self):
        return len(self.items)

    def __repr__(self):
        return f"CSet({set(self.items)!r})"


class Record:
    """Cedar Record: string-keyed map, structural equality."""

    __slots__ = ("m", "_h")

    def __init__(self, m: Optional[Dict[str, Any]] = None):
        self.m = dict(m or {})
        self._h = None

    def __eq__(self, o):
        return isinstance(o, Record) and o.m == self.m

    def __hash__(self):
        if self._h is None:
            self._h = hash(("R", frozenset(self.m.items())))
        return self._h

    def __repr__(self):
        return f"Record({self.m!r})"


class Decimal:
    """Cedar decimal: fixed point, 4 fractional digits, int64 range."""

    __slots__ = ("v",)

    def __init__(self, v: int):
        self.v = v

    def __eq__(self, o):
        return isinstance(o, Decimal) and o.v == self.v

    def __hash__(self):
        return hash(("D", self.v))


class IPAddr:
    __slots__ = ("net",)

    def __init__(self, net):
        self.net = net

    def __eq__(self, o):
        return isinstance(o, IPAddr) and o.net == self.net

    def __hash__(self):
        return hash(("I", self.net))


def type_name(v) -> str:
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, Long):
        return "long"
    if isinstance(v, str):
        return "string"
    if isinstance(v, EntityUID):
        return "entity"
    if isinstance(v, CSet):
        return "set"
    if isinstance(v, Record):
        return "record"
    if isinstance(v, Decimal):
        return "decimal"
    if isinstance(v, IPAddr):
        return "IP"
    return "unknown"


class EvalError(Exception):
    """A Cedar evaluation error. ``kind`` is a stable code shared with the GPU result format."""

    def __init__(self, kind: str, msg: str):
        super().__init__(msg)
        self.kind = kind
        self.msg = msg


def type_error(expected: str, got) -> EvalError:
    return EvalError("type", f"type error: expected {expected}, got {type_name(got)}")


# ----------------------------------------------------------------------------------------------
# Go-compatible JSON helpers (encoding/json HTML-escapes <, >, & and U+2028/9)
# ----------------------------------------------------------------------------------------------

def go_json_string(s: str) -> str:
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif o < 0x20 or ch in "<>&" or o in (0x2028, 0x2029):
            out.append("\\u%04x" % o)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def go_quote(s: str) -> str:
    """Entity-ID quoting used in error messages (escapes only backslash and double quote).
    Error message text is not pinned by any reference test (parity unpinned)."""
    return '"' + s.replace("\\", "\\\\").replace('"', '\\"') + '"'


# ----------------------------------------------------------------------------------------------
# Lexer
# ----------------------------------------------------------------------------------------------

@dataclass
class Tok:
    kind: str  # IDENT, STR, INT, OP, EOF
    text: str
    offset: int
    line: int
    col: int


class ParseError(Exception):
    pass


_OPS3 = ()
_OPS2 = ("==", "!=", "<=", ">=", "&&", "||", "::")
_OPS1 = "()[]{},;.@<>!+-*:"


def tokenize(src: str) -> List[Tok]:
    toks: List[Tok] = []
    b = src.encode("utf-8")
    i, n = 0, len(src)
    line, col = 1, 1
    # offsets are byte offsets; columns are character counts (text/scanner convention)
    boff = 0

    def adv(k):
        nonlocal i, line, col, boff
        for _ in range(k):
            ch = src[i]
            boff += len(ch.encode("utf-8"))
            i += 1
            if ch == "\n":
                line += 1
                col = 1
            else:
                col += 1

    while i < n:
        ch = src[i]
        if ch in " \t\r\n\f\v":
            adv(1)
            continue
        if src.startswith("//", i):
            while i < n and src[i] != "\n":
                adv(1)
            continue
        start = (boff, line, col)
        if ch.isalpha() or ch == "_":
            j = i
            while j < n and (src[j].isalnum() or src[j] == "_"):
                j += 1
            text = src[i:j]
            adv(j - i)
            toks.append(Tok("IDENT", text, *start))
            continue
        if ch.isdigit():
            j = i
            while j < n and src[j].isdigit():
                j += 1
            text = src[i:j]
            adv(j - i)
            toks.append(Tok("INT", text, *start))
            continue
        if ch == '"':
            j = i + 1
            while j < n and src[j] != '"':
                if src[j] == "\\":
                    j += 1
                j += 1
            if j >= n:
                raise ParseError(f"unterminated string at line {line}")
            raw = src[i + 1:j]
            adv(j + 1 - i)
            toks.append(Tok("STR", raw, *start))
            continue
        two = src[i:i + 2]
        if two in _OPS2:
            adv(2)
            toks.append(Tok("OP", two, *start))
            continue
        if ch in _OPS1:
            adv(1)
            toks.append(Tok("OP", ch, *start))
            continue
        raise ParseError(f"unexpected character {ch!r} at line {line} column {col}")
    toks.append(Tok("EOF", "", boff, line, col))
    return toks


def unescape(raw: str, pattern: bool = False):
    """Cedar string escapes. For patterns returns a list of ('lit', str) / ('star',) pieces."""
    out: List[Any] = []
    lit: List[str] = []
    i = 0
    while i < len(raw):
        ch = raw[i]
        if ch == "\\":
            i += 1
            if i >= len(raw):
                raise ParseError("bad escape")
            e = raw[i]
            if e == "n":
                lit.append("\n")
            elif e == "r":
                lit.append("\r")
            elif e == "t":
                lit.append("\t")
            elif e == "\\":
                lit.append("\\")
            elif e == "0":
                lit.append("\0")
            elif e == "'":
                lit.append("'")
            elif e == '"':
                lit.append('"')
            elif e == "*" and pattern:
                lit.append("*")
            elif e == "x":
                h = raw[i + 1:i + 3]
                if len(h) != 2 or int(h, 16) > 0x7F:
                    raise ParseError("bad \\x escape")
                lit.append(chr(int(h, 16)))
                i += 2
            elif e == "u":
                if raw[i + 1:i + 2] != "{":
                    raise ParseError("bad \\u escape")
                j = raw.index("}", i)
                lit.append(chr(int(raw[i + 2:j], 16)))
                i = j
            else:
                raise ParseError(f"bad escape \\{e}")
            i += 1
            continue
        if ch == "*" and pattern:
            if lit:
                out.append(("lit", "".join(lit)))
                lit = []
            out.append(("star",))
            i += 1
            continue
        lit.append(ch)
        i += 1
    if pattern:
        if lit:
            out.append(("lit", "".join(lit)))
        return out
    return "".join(lit)


# ----------------------------------------------------------------------------------------------
# AST
# ----------------------------------------------------------------------------------------------
# Expressions are tuples: (op, *args)
#   ('lit', value) ('var', name) ('and', a, b) ('or', a, b) ('not', a) ('neg', a)
#   ('if', c, t, e) ('bin', op, a, b)  op in == != < <= > >= + - * in
#   ('has', a, key) ('like', a, pattern) ('is', a, type, in_expr|None) ('attr', a, key)
#   ('call', fname, args) ('method', a, name, args) ('set', [e...]) ('rec', [(k, e)...])


@dataclass
class Scope:
    kind: str  # any, eq, in, is, isin, inset
    etype: Optional[str] = None
    entity: Optional[EntityUID] = None
    entities: Optional[List[EntityUID]] = None


@dataclass
class Policy:
    effect: str
    principal: Scope
    action: Scope
    resource: Scope
    conditions: List[Tuple[str, Any]]
    annotations: Dict[str, str]
    offset: int
    line: int
    col: int
    filename: str = ""
    pid: str = ""


RESERVED = {"true", "false", "if", "then", "else", "in", "is", "like", "has", "__cedar"}


class Parser:
    def __init__(self, src: str, filename: str = ""):
        self.toks = tokenize(src)
        self.i = 0
        self.filename = filename

    def peek(self, k=0) -> Tok:
        return self.toks[min(self.i + k, len(self.toks) - 1)]

    def next(self) -> Tok:
        t = self.toks[self.i]
        self.i += 1
        return t

    def expect(self, text: str) -> Tok:
        t = self.next()
        if t.text != text or t.kind not in ("OP", "IDENT"):
            raise ParseError(f"{self.filename}:{t.line}:{t.col}: expected {text!r}, got {t.text!r}")
        return t

    def is_op(self, text: str, k=0) -> bool:
        t = self.peek(k)
        return t.kind == "OP" and t.text == text

    def is_kw(self, text: str, k=0) -> bool:
        t = self.peek(k)
        return t.kind == "IDENT" and t.text == text

    # --- policies -------------------------------------------------------------------------
    def policies(self) -> List[Policy]:
        out = []
        while self.peek().kind != "EOF":
            out.append(self.policy())
        return out

    def policy(self) -> Policy:
        first = self.peek()
        ann: Dict[str, str] = {}
        while self.is_op("@"):
            self.next()
            name = self.next()
            if name.kind != "IDENT":
                raise ParseError("bad annotation")
            val = ""
            if self.is_op("("):
                self.next()
                s = self.next()
                if s.kind != "STR":
                    raise ParseError("annotation value must be a string")
                val = unescape(s.text)
                self.expect(")")
            if name.text in ann:
                raise ParseError(f"duplicate annotation @{name.text}")
            ann[name.text] = val
        eff = self.next()
        if eff.kind != "IDENT" or eff.text not in ("permit", "forbid"):
            raise ParseError(f"{self.filename}:{eff.line}:{eff.col}: expected permit or forbid, got {eff.text!r}")
        self.expect("(")
        p = self.scope("principal")
        self.expect(",")
        a = self.action_scope()
        self.expect(",")
        r = self.scope("resource")
        self.expect(")")
        conds = []
        while self.is_kw("when") or self.is_kw("unless"):
            kind = self.next().text
            self.expect("{")
            e = self.expr()
            self.expect("}")
            conds.append((kind, e))
        self.expect(";")
        return Policy(eff.text, p, a, r, conds, ann, first.offset, first.line, first.col, self.filename)

    def path(self) -> str:
        t = self.next()
        if t.kind != "IDENT":
            raise ParseError(f"expected identifier, got {t.text!r}")
        parts = [t.text]
        while self.is_op("::") and self.peek(1).kind == "IDENT":
            self.next()
            parts.append(self.next().text)
        return "::".join(parts)

    def entity_ref(self) -> EntityUID:
        t = self.next()
        if t.kind != "IDENT":
            raise ParseError(f"expected entity, got {t.text!r}")
        parts = [t.text]
        while True:
            self.expect("::")
            n = self.next()
            if n.kind == "STR":
                return EntityUID("::".join(parts), unescape(n.text))
            if n.kind != "IDENT":
                raise ParseError("bad entity reference")
            parts.append(n.text)

    def scope(self, var: str) -> Scope:
        self.expect(var)
        if self.is_op("=="):
            self.next()
            return Scope("eq", entity=self.entity_ref())
        if self.is_kw("is"):
            self.next()
            t = self.path()
            if self.is_kw("in"):
                self.next()
                return Scope("isin", etype=t, entity=self.entity_ref())
            return Scope("is", etype=t)
        if self.is_kw("in"):
            self.next()
            return Scope("in", entity=self.entity_ref())
        return Scope("any")

    def action_scope(self) -> Scope:
        self.expect("action")
        if self.is_op("=="):
            self.next()
            return Scope("eq", entity=self.entity_ref())
        if self.is_kw("in"):
            self.next()
            if self.is_op("["):
                self.next()
                ents = []
                if not self.is_op("]"):
                    ents.append(self.entity_ref())
                    while self.is_op(","):
                        self.next()
                        if self.is_op("]"):
                            break
                        ents.append(self.entity_ref())
                self.expect("]")
                return Scope("inset", entities=ents)
            return Scope("in", entity=self.entity_ref())
        return Scope("any")

    # --- expressions ----------------------------------------------------------------------
    def expr(self):
        if self.is_kw("if"):
            self.next()
            c = self.expr()
            self.expect("then")
            t = self.expr()
            self.expect("else")
            e = self.expr()
            return ("if", c, t, e)
        return self.or_()

    def or_(self):
        lhs = self.and_()
        while self.is_op("||"):
            self.next()
            lhs = ("or", lhs, self.and_())
        return lhs

    def and_(self):
        lhs = self.relation()
        while self.is_op("&&"):
            self.next()
            lhs = ("and", lhs, self.relation())
        return lhs

    def relation(self):
        lhs = self.add()
        t = self.peek()
        if t.kind == "OP" and t.text in ("==", "!=", "<", "<=", ">", ">="):
            self.next()
            return ("bin", t.text, lhs, self.add())
        if self.is_kw("in"):
            self.next()
            return ("bin", "in", lhs, self.add())
        if self.is_kw("has"):
            self.next()
            k = self.next()
            if k.kind == "STR":
                return ("has", lhs, unescape(k.text))
            if k.kind != "IDENT":
                raise ParseError("expected attribute after has")
            return ("has", lhs, k.text)
        if self.is_kw("like"):
            self.next()
            s = self.next()
            if s.kind != "STR":
                raise ParseError("expected pattern after like")
            return ("like", lhs, tuple(tuple(x) for x in unescape(s.text, pattern=True)))
        if self.is_kw("is"):
            self.next()
            ty = self.path()
            inx = None
            if self.is_kw("in"):
                self.next()
                inx = self.add()
            return ("is", lhs, ty, inx)
        return lhs

    def add(self):
        lhs = self.mult()
        while self.is_op("+") or self.is_op("-"):
            op = self.next().text
            lhs = ("bin", op, lhs, self.mult())
        return lhs

    def mult(self):
        lhs = self.unary()
        while self.is_op("*"):
            self.next()
            lhs = ("bin", "*", lhs, self.unary())
        return lhs

    def unary(self):
        ops = []
        while self.is_op("!") or self.is_op("-"):
            ops.append(self.next().text)
        if len(ops) > 4:
            raise ParseError("too many unary operators")
        # a '-' directly before an integer literal folds into the literal (allows LONG_MIN)
        if ops and ops[-1] == "-" and self.peek().kind == "INT":
            ops.pop()
            v = -int(self.next().text)
            if v < LONG_MIN:
                raise ParseError("integer literal out of range")
            e = self.member_tail(("lit", Long(v)))
        else:
            e = self.member()
        for op in reversed(ops):
            e = ("not", e) if op == "!" else ("neg", e)
        return e

    def member(self):
        return self.member_tail(self.primary())

    def member_tail(self, e):
        while True:
            if self.is_op("."):
                self.next()
                name = self.next()
                if name.kind != "IDENT":
                    raise ParseError("expected attribute name")
                if self.is_op("("):
                    self.next()
                    args = self.expr_list(")")
                    want = _METHOD_ARITY.get(name.text)
                    if want is None:
                        raise ParseError(f"`{name.text}` is not a method")
                    if len(args) != want:
                        raise ParseError(f"{name.text} expects {want} argument(s)")
                    e = ("method", e, name.text, args)
                else:
                    e = ("attr", e, name.text)
            elif self.is_op("["):
                self.next()
                s = self.next()
                if s.kind != "STR":
                    raise ParseError("expected string index")
                self.expect("]")
                e = ("attr", e, unescape(s.text))
            else:
                return e

    def expr_list(self, close: str):
        args = []
        if not self.is_op(close):
            args.append(self.expr())
            while self.is_op(","):
                self.next()
                if self.is_op(close):
                    break
                args.append(self.expr())
        self.expect(close)
        return args

    def primary(self):
        t = self.peek()
        if t.kind == "INT":
            self.next()
            v = int(t.text)
            if v > LONG_MAX:
                raise ParseError("integer literal out of range")
            return ("lit", Long(v))
        if t.kind == "STR":
            self.next()
            return ("lit", unescape(t.text))
        if t.kind == "OP" and t.text == "(":
            self.next()
            e = self.expr()
            self.expect(")")
            return e
        if t.kind == "OP" and t.text == "[":
            self.next()
            return ("set", self.expr_list("]"))
        if t.kind == "OP" and t.text == "{":
            self.next()
            items = []
            seen = set()
            if not self.is_op("}"):
                while True:
                    k = self.next()
                    if k.kind == "STR":
                        key = unescape(k.text)
                    elif k.kind == "IDENT":
                        key = k.text
                    else:
                        raise ParseError("bad record key")
                    if key in seen:
                        raise ParseError(f"duplicate record key {key!r}")
                    seen.add(key)
                    self.expect(":")
                    items.append((key, self.expr()))
                    if self.is_op(","):
                        self.next()
                        if self.is_op("}"):
                            break
                        continue
                    break
            self.expect("}")
            return ("rec", items)
        if t.kind == "IDENT":
            if t.text == "true":
                self.next()
                return ("lit", True)
            if t.text == "false":
                self.next()
                return ("lit", False)
            if t.text in ("principal", "action", "resource", "context") and not self.is_op("::", 1):
                self.next()
                return ("var", t.text)
            # entity reference or extension function call
            j = 1
            while self.is_op("::", j) and self.peek(j + 1).kind == "IDENT":
                j += 2
            if self.is_op("::", j) and self.peek(j + 1).kind == "STR":
                return ("lit", self.entity_ref())
            if self.is_op("(", j):
                name = self.path()
                if name not in ("ip", "decimal"):
                    raise ParseError(f"`{name}` is not a function")
                self.expect("(")
                args = self.expr_list(")")
                if len(args) != 1:
                    raise ParseError(f"{name} expects 1 argument")
                return ("call", name, args)
            raise ParseError(f"{self.filename}:{t.line}:{t.col}: unexpected identifier {t.text!r}")
        raise ParseError(f"{self.filename}:{t.line}:{t.col}: unexpected token {t.text!r}")


# Cedar's extension functions are ip/decimal (one argument each); its methods and their argument
# counts are below. Other names or counts are parse errors (the device compiler's parser.cpp
# rejects them the same way), so the whole document is rejected or skipped.
_METHOD_ARITY = {"contains": 1, "containsAll": 1, "containsAny": 1, "lessThan": 1, "lessThanOrEqual": 1,
                 "greaterThan": 1, "greaterThanOrEqual": 1, "isInRange": 1,
                 "isEmpty": 0, "isIpv4": 0, "isIpv6": 0, "isLoopback": 0, "isMulticast": 0}


def parse_policies(src: str, filename: str = "") -> List[Policy]:
    return Parser(src, filename).policies()


# ----------------------------------------------------------------------------------------------
# Extension types
# ----------------------------------------------------------------------------------------------

def parse_decimal(s: str) -> Decimal:
    neg = s.startswith("-")
    body = s[1:] if neg else s
    if "." not in body:
        raise EvalError("extension", f"error parsing decimal value: {s}")
    ip, fp = body.split(".", 1)
    if not (ip.isascii() and ip.isdigit() and fp.isascii() and fp.isdigit()) or len(fp) > 4:
        raise EvalError("extension", f"error parsing decimal value: {s}")
    v = int(ip) * 10000 + int(fp.ljust(4, "0"))
    if neg:
        v = -v
    if v < LONG_MIN or v > LONG_MAX:
        raise EvalError("extension", f"error parsing decimal value: {s}")
    return Decimal(v)


def parse_ip(s: str) -> IPAddr:
    # netip.ParsePrefix / ParseAddr rules where Python's ipaddress is looser: the prefix length is
    # decimal digits without a leading zero (no netmask form), and IPv6 zones are not addresses
    addr, slash, bits = s.partition("/")
    if "%" in addr or (slash and not re.fullmatch(r"0|[1-9][0-9]{0,2}", bits)):
        raise EvalError("extension", f"error parsing ip value: {s}")
    try:
        if "/" in s:
            net = ipaddress.ip_network(s, strict=False)
            # Cedar keeps the host bits; prefix semantics via network for containment
            addr = ipaddress.ip_interface(s)
            return IPAddr(addr)
        return IPAddr(ipaddress.ip_interface(s))
    except ValueError:
        raise EvalError("extension", f"error parsing ip value: {s}")


# ----------------------------------------------------------------------------------------------
# Entities and requests
# ----------------------------------------------------------------------------------------------

@dataclass
class Entity:
    uid: EntityUID
    attrs: Record = field(default_factory=Record)
    parents: Tuple[EntityUID, ...] = ()


EntityMap = Dict[EntityUID, Entity]


@dataclass
class Request:
    principal: EntityUID
    action: EntityUID
    resource: EntityUID
    context: Record = field(default_factory=Record)


def merge_static_entities(em: EntityMap, static: Optional[EntityMap]) -> EntityMap:
    """The EntityMap a request is evaluated against when the policy image carries static entities
    (a group / namespace hierarchy the request does not hold; cedargpu.h cg_compiler_set_entities).
    This is what a maintainer merging a static entity source into the map built by
    RecordToCedarResource (authorizer.go:89-111) before TieredPolicyStores.IsAuthorized
    (store.go:25) would hand cedar-go: the request's entities, plus every static entity the request
    lacks; for a UID in both, the request's attributes and the union of both parent lists."""
    if not static:
        return em
    out = dict(em)
    for uid, se in static.items():
        e = out.get(uid)
        if e is None:
            out[uid] = se
        else:
            out[uid] = Entity(uid, e.attrs, tuple(dict.fromkeys(tuple(e.parents) + tuple(se.parents))))
    return out


def ancestors(em: EntityMap, uid: EntityUID) -> set:
    seen = set()
    stack = [uid]
    while stack:
        u = stack.pop()
        e = em.get(u)
        if e is None:
            continue
        for p in e.parents:
            if p not in seen:
                seen.add(p)
                stack.append(p)
    return seen


def entity_in(em: EntityMap, a: EntityUID, b: EntityUID) -> bool:
    return a == b or b in ancestors(em, a)


# ----------------------------------------------------------------------------------------------
# Evaluator
# ----------------------------------------------------------------------------------------------

def _check_long(v: int) -> Long:
    if v < LONG_MIN or v > LONG_MAX:
        raise EvalError("overflow", "integer overflow")
    return Long(v)


def like_match(s: str, pat) -> bool:
    # classic greedy glob with backtracking over pieces
    pieces = list(pat)

    def rec(si: int, pi: int) -> bool:
        while pi < len(pieces):
            p = pieces[pi]
            if p[0] == "lit":
                if not s.startswith(p[1], si):
                    return False
                si += len(p[1])
                pi += 1
            else:
                # star: try every split point
                if pi == len(pieces) - 1:
                    return True
                for k in range(si, len(s) + 1):
                    if rec(k, pi + 1):
                        return True
                return False
        return si == len(s)

    return rec(0, 0)


class Evaluator:
    def __init__(self, em: EntityMap, req: Request):
        self.em = em
        self.req = req

    def as_bool(self, v):
        if not isinstance(v, bool):
            raise type_error("bool", v)
        return v

    def ev(self, e):
        op = e[0]
        if op == "lit":
            return e[1]
        if op == "var":
            n = e[1]
            if n == "principal":
                return self.req.principal
            if n == "action":
                return self.req.action
            if n == "resource":
                return self.req.resource
            return self.req.context
        if op == "and":
            if not self.as_bool(self.ev(e[1])):
                return False
            return self.as_bool(self.ev(e[2]))
        if op == "or":
            if self.as_bool(self.ev(e[1])):
                return True
            return self.as_bool(self.ev(e[2]))
        if op == "not":
            return not self.as_bool(self.ev(e[1]))
        if op == "neg":
            v = self.ev(e[1])
            if not isinstance(v, Long):
                raise type_error("long", v)
            return _check_long(-v.v)
        if op == "if":
            c = self.as_bool(self.ev(e[1]))
            return self.ev(e[2]) if c else self.ev(e[3])
        if op == "bin":
            return self.binop(e[1], self.ev(e[2]), self.ev(e[3]))
        if op == "has":
            v = self.ev(e[1])
            if isinstance(v, EntityUID):
                ent = self.em.get(v)
                return ent is not None and e[2] in ent.attrs.m
            if isinstance(v, Record):
                return e[2] in v.m
            raise type_error("entity or record", v)
        if op == "attr":
            v = self.ev(e[1])
            key = e[2]
            if isinstance(v, EntityUID):
                ent = self.em.get(v)
                if ent is None:
                    raise EvalError("entity_not_found", f"entity `{v}` does not exist")
                if key not in ent.attrs.m:
                    raise EvalError("attr_missing", f"`{v}` does not have the attribute `{key}`")
                return ent.attrs.m[key]
            if isinstance(v, Record):
                if key not in v.m:
                    raise EvalError("attr_missing", f"record does not have the attribute `{key}`")
                return v.m[key]
            raise type_error("entity or record", v)
        if op == "like":
            v = self.ev(e[1])
            if not isinstance(v, str):
                raise type_error("string", v)
            return like_match(v, e[2])
        if op == "is":
            v = self.ev(e[1])
            if not isinstance(v, EntityUID):
                raise type_error("entity", v)
            if v.type != e[2]:
                return False
            if e[3] is None:
                return True
            return self.in_op(v, self.ev(e[3]))
        if op == "set":
            return CSet([self.ev(x) for x in e[1]])
        if op == "rec":
            return Record({k: self.ev(x) for k, x in e[1]})
        if op == "call":
            return self.call(e[1], [self.ev(x) for x in e[2]])
        if op == "method":
            recv = self.ev(e[1])
            return self.method(recv, e[2], [self.ev(x) for x in e[3]])
        raise AssertionError(op)

    def in_op(self, a, b):
        if not isinstance(a, EntityUID):
            raise type_error("entity", a)
        if isinstance(b, EntityUID):
            return entity_in(self.em, a, b)
        if isinstance(b, CSet):
            anc = None
            for x in b:
                if not isinstance(x, EntityUID):
                    raise type_error("entity", x)
            for x in b:
                if x == a:
                    return True
                if anc is None:
                    anc = ancestors(self.em, a)
                if x in anc:
                    return True
            return False
        raise type_error("set or entity", b)

    def binop(self, op, a, b):
        if op == "==":
            return a == b
        if op == "!=":
            return a != b
        if op == "in":
            return self.in_op(a, b)
        if op in ("<", "<=", ">", ">="):
            if not isinstance(a, Long):
                raise type_error("long", a)
            if not isinstance(b, Long):
                raise type_error("long", b)
            x, y = a.v, b.v
            return {"<": x < y, "<=": x <= y, ">": x > y, ">=": x >= y}[op]
        if op in ("+", "-", "*"):
            if not isinstance(a, Long):
                raise type_error("long", a)
            if not isinstance(b, Long):
                raise type_error("long", b)
            x, y = a.v, b.v
            r = x + y if op == "+" else (x - y if op == "-" else x * y)
            return _check_long(r)
        raise AssertionError(op)

    def call(self, name, args):
        if len(args) != 1 or not isinstance(args[0], str):
            raise EvalError("extension", f"{name} takes one string argument")
        if name == "decimal":
            return parse_decimal(args[0])
        if name == "ip":
            return parse_ip(args[0])
        raise EvalError("extension", f"unknown extension function {name}")

    def method(self, recv, name, args):
        if name in ("contains", "containsAll", "containsAny"):
            if not isinstance(recv, CSet):
                raise type_error("set", recv)
            if len(args) != 1:
                raise EvalError("arity", f"{name} takes one argument")
            if name == "contains":
                return args[0] in recv.items
            other = args[0]
            if not isinstance(other, CSet):
                raise type_error("set", other)
            if name == "containsAll":
                return other.items <= recv.items
            return len(other.items & recv.items) > 0
        if name == "isEmpty":
            if not isinstance(recv, CSet):
                raise type_error("set", recv)
            return len(recv.items) == 0
        if name in ("lessThan", "lessThanOrEqual", "greaterThan", "greaterThanOrEqual"):
            if not isinstance(recv, Decimal):
                raise type_error("decimal", recv)
            o = args[0] if args else None
            if not isinstance(o, Decimal):
                raise type_error("decimal", o)
            x, y = recv.v, o.v
            return {"lessThan": x < y, "lessThanOrEqual": x <= y,
                    "greaterThan": x > y, "greaterThanOrEqual": x >= y}[name]
        if name in ("isIpv4", "isIpv6", "isLoopback", "isMulticast", "isInRange"):
            if not isinstance(recv, IPAddr):
                raise type_error("IP", recv)
            ip = recv.net
            if name == "isIpv4":
                return ip.version == 4
            if name == "isIpv6":
                return ip.version == 6
            if name == "isLoopback":
                return ip.ip.is_loopback
            if name == "isMulticast":
                return ip.ip.is_multicast
            o = args[0] if args else None
            if not isinstance(o, IPAddr):
                raise type_error("IP", o)
            if o.net.version != ip.version:
                return False
            return ip.network.subnet_of(o.net.network) if ip.network.prefixlen >= o.net.network.prefixlen else False
        raise EvalError("unknown_method", f"unknown method {name}")


def scope_match(ev: Evaluator, sc: Scope, v: EntityUID) -> bool:
    if sc.kind == "any":
        return True
    if sc.kind == "eq":
        return v == sc.entity
    if sc.kind == "in":
        return entity_in(ev.em, v, sc.entity)
    if sc.kind == "is":
        return v.type == sc.etype
    if sc.kind == "isin":
        return v.type == sc.etype and entity_in(ev.em, v, sc.entity)
    if sc.kind == "inset":
        anc = ancestors(ev.em, v)
        return any(x == v or x in anc for x in sc.entities)
    raise AssertionError(sc.kind)


def eval_policy(p: Policy, ev: Evaluator) -> bool:
    """Returns satisfied? Raises EvalError on error (policy skipped by the authorizer)."""
    if not scope_match(ev, p.principal, ev.req.principal):
        return False
    if not scope_match(ev, p.action, ev.req.action):
        return False
    if not scope_match(ev, p.resource, ev.req.resource):
        return False
    for kind, e in p.conditions:
        v = ev.as_bool(ev.ev(e))
        if kind == "when" and not v:
            return False
        if kind == "unless" and v:
            return False
    return True


# ----------------------------------------------------------------------------------------------
# PolicySet / Diagnostic / tiers
# ----------------------------------------------------------------------------------------------

@dataclass
class DiagReason:
    policy: str
    filename: str
    offset: int
    line: int
    column: int
    index: int = 0


@dataclass
class DiagError:
    policy: str
    filename: str
    offset: int
    line: int
    column: int
    message: str
    kind: str = ""
    index: int = 0


@dataclass
class Diagnostic:
    reasons: List[DiagReason] = field(default_factory=list)
    errors: List[DiagError] = field(default_factory=list)

    def to_go_json(self) -> str:
        """json.Marshal(cedar.Diagnostic) with omitempty slices."""
        parts = []
        if self.reasons:
            parts.append('"reasons":[' + ",".join(_reason_json(r) for r in self.reasons) + "]")
        if self.errors:
            parts.append('"errors":[' + ",".join(_error_json(e) for e in self.errors) + "]")
        return "{" + ",".join(parts) + "}"

    def reasons_json(self) -> str:
        """json.Marshal(diagnostics.Reasons) (admission handler.go:64-66)."""
        return "[" + ",".join(_reason_json(r) for r in self.reasons) + "]"


def _pos_json(filename, offset, line, column):
    return ('{"filename":' + go_json_string(filename) + f',"offset":{offset},"line":{line},"column":{column}' + "}")


def _reason_json(r: DiagReason) -> str:
    return '{"policy":' + go_json_string(r.policy) + ',"position":' + _pos_json(r.filename, r.offset, r.line, r.column) + "}"


def _error_json(e: DiagError) -> str:
    return ('{"policy":' + go_json_string(e.policy) + ',"position":' + _pos_json(e.filename, e.offset, e.line, e.column)
            + ',"message":' + go_json_string(e.message) + "}")


class PolicySet:
    """cedar.PolicySet restatement; policies kept in insertion order (see module docstring)."""

    def __init__(self):
        self.policies: List[Policy] = []
        self.ids: Dict[str, int] = {}

    def add(self, pid: str, p: Policy):
        if pid in self.ids:
            self.policies[self.ids[pid]] = p
            p.pid = pid
            return
        p.pid = pid
        self.ids[pid] = len(self.policies)
        self.policies.append(p)

    def remove(self, pid: str):
        if pid not in self.ids:
            return
        self.policies = [p for p in self.policies if p.pid != pid]
        self.ids = {p.pid: i for i, p in enumerate(self.policies)}

    @staticmethod
    def from_bytes(filename: str, src: str) -> "PolicySet":
        """cedar.NewPolicySetFromBytes: IDs policy0, policy1, ... (memory.go:18)."""
        ps = PolicySet()
        for i, p in enumerate(parse_policies(src, filename)):
            ps.add(f"policy{i}", p)
        return ps

    def is_authorized(self, em: EntityMap, req: Request) -> Tuple[bool, Diagnostic]:
        ev = Evaluator(em, req)
        forbids, permits, errors = [], [], []
        for idx, p in enumerate(self.policies):
            try:
                sat = eval_policy(p, ev)
            except EvalError as err:
                errors.append(DiagError(p.pid, p.filename, p.offset, p.line, p.col,
                                        f"while evaluating policy `{p.pid}`: {err.msg}", err.kind, idx))
                continue
            if not sat:
                continue
            r = DiagReason(p.pid, p.filename, p.offset, p.line, p.col, idx)
            (forbids if p.effect == "forbid" else permits).append(r)
        if forbids:
            return False, Diagnostic(forbids, errors)
        if permits:
            return True, Diagnostic(permits, errors)
        return False, Diagnostic([], errors)


def tiered_is_authorized(tiers: List[PolicySet], em: EntityMap, req: Request) -> Tuple[bool, Diagnostic, int]:
    """TieredPolicyStores.IsAuthorized (store.go:25-42). Also returns the deciding tier index."""
    decision, diag = False, Diagnostic()
    t = 0
    for t, ps in enumerate(tiers):
        decision, diag = ps.is_authorized(em, req)
        if t == len(tiers) - 1:
            break
        if (not decision) and not diag.reasons and not diag.errors:
            continue
        break
    return decision, diag, t


# ----------------------------------------------------------------------------------------------
# Cedar JSON (entities / values / requests) — the format shared with the C-ABI test entry points
# ----------------------------------------------------------------------------------------------

def value_from_json(j):
    if isinstance(j, bool):
        return j
    if isinstance(j, int):
        return Long(j)
    if isinstance(j, str):
        return j
    if isinstance(j, list):
        return CSet([value_from_json(x) for x in j])
    if isinstance(j, dict):
        if "__entity" in j and len(j) == 1:
            return EntityUID(j["__entity"]["type"], j["__entity"]["id"])
        if "__extn" in j and len(j) == 1:
            fn, arg = j["__extn"]["fn"], j["__extn"]["arg"]
            return parse_decimal(arg) if fn == "decimal" else parse_ip(arg)
        return Record({k: value_from_json(v) for k, v in j.items()})
    raise ValueError(f"bad value json {j!r}")


def value_to_json(v):
    if isinstance(v, bool) or isinstance(v, str):
        return v
    if isinstance(v, Long):
        return v.v
    if isinstance(v, EntityUID):
        return {"__entity": {"type": v.type, "id": v.id}}
    if isinstance(v, CSet):
        return [value_to_json(x) for x in v]
    if isinstance(v, Record):
        return {k: value_to_json(x) for k, x in v.m.items()}
    if isinstance(v, IPAddr):
        return {"__extn": {"fn": "ip", "arg": str(v.net)}}
    if isinstance(v, Decimal):
        sign = "-" if v.v < 0 else ""
        a = abs(v.v)
        return {"__extn": {"fn": "decimal", "arg": f"{sign}{a // 10000}.{a % 10000:04d}"}}
    raise ValueError(v)


def uid_from_json(j) -> EntityUID:
    if "__entity" in j:
        j = j["__entity"]
    return EntityUID(j["type"], j["id"])


def entities_from_json(arr) -> EntityMap:
    em: EntityMap = {}
    for e in arr:
        uid = uid_from_json(e["uid"])
        attrs = value_from_json(e.get("attrs", {}))
        parents = tuple(uid_from_json(p) for p in e.get("parents", []))
        em[uid] = Entity(uid, attrs, parents)
    return em


def entities_to_json(em: EntityMap):
    out = []
    for e in em.values():
        out.append({"uid": {"type": e.uid.type, "id": e.uid.id},
                    "attrs": value_to_json(e.attrs),
                    "parents": [{"type": p.type, "id": p.id} for p in e.parents]})
    return out


def request_from_json(j) -> Request:
    return Request(uid_from_json(j["principal"]), uid_from_json(j["action"]), uid_from_json(j["resource"]),
                   value_from_json(j.get("context", {})))


def request_to_json(r: Request):
    return {"principal": {"type": r.principal.type, "id": r.principal.id},
            "action": {"type": r.action.type, "id": r.action.id},
            "resource": {"type": r.resource.type, "id": r.resource.id},
            "context": value_to_json(r.context)}

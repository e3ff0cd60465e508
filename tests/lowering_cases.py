"""Valid Cedar that the device compiler once rejected (round-1 VERDICT: "lower the rejected-but-valid
shapes"): ip()/decimal() of runtime strings, expressions deeper than the 8 register slots, set and
record literals beyond the private lane array, and policy records larger than one 16 KiB LDS chunk.
Each case is (store texts, items); tests compare the device with the oracles on them."""
import random

IPS = ["10.1.2.3", "10.0.0.0/8", "10.0.0.1/8", "127.0.0.1", "224.0.0.5", "::1", "::1/128", "fe80::/10",
       "::ffff:10.0.0.1", "2001:db8::8a2e:370:7334", "0.0.0.0/0", "255.255.255.255", "ff02::1", "::",
       "1:2:3:4:5:6:7::", "192.168.1.1/32",
       # invalid
       "", "1.2.3", "1.2.3.4.5", "01.2.3.4", "256.1.1.1", "1.2.3.4/33", "::1/129", "1:2:3:4:5:6:7:8:9",
       "1::2::3", "abc", "1.2.3.4/", "g::1", "1.2.3.4/024", "1.2.3.4/255.0.0.0", "fe80::1%eth0", " 1.2.3.4",
       "1.2.3.4/8/8", "::1:", ":1::", "12345::", "1.2.3.4:80"]
DECS = ["1.5", "-0.0001", "922337203685477.5807", "-922337203685477.5808", "12.3", "0.0", "2.5", "2.4999",
        # invalid
        "1", ".5", "1.", "1.23456", "922337203685477.5808", "-922337203685477.5809", "abc", "+1.0", "1.2.3",
        "", "-", "--1.0", "1e3", "١.٠", "99999999999999999999.0"]

EXT_POLICIES = """
permit (principal, action, resource) when { ip(context.s).isIpv4() };
permit (principal, action, resource) when { ip(context.s).isInRange(ip("10.0.0.0/8")) };
forbid (principal, action, resource) when { ip(context.s) == ip("::1") } unless { context.n == 7 };
permit (principal, action, resource) when { decimal(context.d).lessThan(decimal("2.5")) };
permit (principal, action, resource) when { decimal(context.d) == decimal("-0.0001") };
permit (principal, action, resource) when { ip(context.s).isLoopback() || ip(context.s).isMulticast() };
permit (principal, action, resource) when { ip(context.n).isIpv6() };
permit (principal, action, resource) when { ip(context.s).isIpv6() && ip("::/0").isInRange(ip(context.s)) };
permit (principal, action, resource) when { decimal(context.d).greaterThanOrEqual(decimal(context.d2)) };
permit (principal, action, resource) when { [ip(context.s), decimal(context.d)].contains(ip("10.1.2.3")) };
"""


def _req(ctx):
    return {"principal": {"type": "User", "id": "u"}, "action": {"type": "Action", "id": "get"},
            "resource": {"type": "Res", "id": "r"}, "context": ctx}


def ext_runtime_case(n=400, seed=0):
    r = random.Random(seed)
    items = []
    for k in range(n):
        ctx = {"s": IPS[k % len(IPS)], "d": DECS[k % len(DECS)], "d2": r.choice(DECS)}
        ctx["n"] = r.choice([7, 3, "::1", "1.2.3.4", True])
        if k % 9 == 0:
            del ctx["s"]  # attribute errors ahead of the parse
        items.append(([], _req(ctx)))
    return [("ext.cedar", EXT_POLICIES)], items


def _chain(depth, r):
    """Right-nested expression: every level holds its left operand in a slot while the right
    one is evaluated, so `depth` levels need depth + 1 slots (the first 8 in registers)."""
    e = r.choice(["context.a", "context.b", str(r.randint(-3, 3))])
    for _ in range(depth):
        op = r.choice(["+", "-", "*", "+", "-"])
        e = f"{r.choice(['context.a', 'context.b', str(r.randint(-3, 3))])} {op} ({e})"
    return e


def _bool_chain(depth, r):
    e = f"context.a < {r.randint(-5, 5)}"
    for _ in range(depth):
        op = r.choice(["&&", "||", "==", "!="])
        left = r.choice(["context.c", f"context.b > {r.randint(-5, 5)}", "true", "context.a == context.b"])
        e = f"({left}) {op} ({e})"
        if r.random() < 0.2:
            e = f"if context.c then ({e}) else (!({e}))" if len(e) < 4000 else e
    return e


def deep_nesting_case(n=300, seed=0):
    r = random.Random(seed)
    pols = []
    for depth in (6, 9, 12, 20, 40, 62):
        pols.append(f"permit (principal, action, resource) when {{ ({_chain(depth, r)}) > 0 }};")
        pols.append(f"forbid (principal, action, resource) when {{ {_bool_chain(depth, r)} }};")
        # nested runtime sets/records held in spilled slots
        s = "context.a"
        for k in range(min(depth, 7)):  # value nesting within the device deep-equality limit
            s = f"[context.b, {s}, {k}]" if k % 2 else f"{{k{k}: {s}, x: context.a}}"
        pols.append(f"permit (principal, action, resource) when {{ {s} == {s} && context.c }};")
    items = []
    for k in range(n):
        ctx = {"a": r.randint(-4, 4), "b": r.randint(-4, 4), "c": r.random() < 0.5}
        if k % 17 == 0:
            ctx["b"] = "str"  # type errors deep in the chains
        if k % 23 == 0:
            ctx["a"] = 9223372036854775807  # overflow
        items.append(([], _req(ctx)))
    return [("deep.cedar", "\n".join(pols))], items


def big_literal_case(n=200, seed=0):
    r = random.Random(seed)
    set100 = ", ".join(str(k) for k in range(99))
    rec100 = ", ".join(f"k{k}: {k}" for k in range(99))
    set1500 = ", ".join(str(3 * k) for k in range(1500))
    pols = [
        f"permit (principal, action, resource) when {{ [context.a, {set100}].contains(context.b) }};",
        f"permit (principal, action, resource) when {{ {{x: context.a, {rec100}}}[\"k77\"] == context.b }};",
        f"forbid (principal, action, resource) when {{ [{set1500}, context.a].contains(context.b + 1000) }};",
        f"permit (principal, action, resource) when {{ {{x: context.a, {rec100}}} == {{x: context.b, {rec100}}} }};",
        f"permit (principal, action, resource) when {{ [context.a, {set100}].containsAll([context.b, 5]) }};",
        "permit (principal, action, resource) when { [" + ", ".join(f"context.a + {k}" for k in range(300)) +
        "].contains(context.b) };",
    ]
    items = []
    for k in range(n):
        ctx = {"a": r.randint(-2, 200), "b": r.randint(-2, 4000)}
        if k % 11 == 0:
            ctx["b"] = ctx["a"]
        if k % 13 == 0:
            del ctx["a"]
        items.append(([], _req(ctx)))
    return [("big.cedar", "\n".join(pols))], items


def big_record_case(n=200, seed=0):
    """Policies whose stream records exceed the 16 KiB LDS chunk: hundreds of `when` clauses
    (flat, so the Python oracle does not recurse deeply), mixed with ordinary policies."""
    r = random.Random(seed)
    pols = ["permit (principal, action, resource) when { context.a > 0 };"]
    for p in range(3):
        clauses = " ".join(f"when {{ context.a + {k} > {r.randint(-50, 5)} && context.b != {k} }}"
                           for k in range(400 + 100 * p))
        eff = "forbid" if p == 1 else "permit"
        pols.append(f"{eff} (principal, action, resource) {clauses};")
        pols.append("permit (principal, action, resource) when { context.b < 3 };")
    items = []
    for k in range(n):
        ctx = {"a": r.randint(-3, 60), "b": r.randint(-3, 500)}
        if k % 7 == 0:
            ctx["b"] = "x"
        items.append(([], _req(ctx)))
    return [("rec.cedar", "\n".join(pols))], items


CASES = {"ext_runtime": ext_runtime_case, "deep_nesting": deep_nesting_case,
         "big_literal": big_literal_case, "big_record": big_record_case}

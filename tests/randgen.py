"""Seeded random Cedar policies + entity maps for differential testing (GPU vs oracle).

Covers every operator the device evaluates: attribute access on entities/records (present,
missing, absent entity), has, ==/!= (incl. deep set/record equality), </<=/>/>=, +,-,* with
overflow, unary -, !, &&/|| short-circuit incl. type errors, if-then-else, in (entity / set /
hierarchy), is / is-in, like (wildcards, escaped star), contains/containsAll/containsAny/isEmpty,
runtime-built sets/records, decimal and ip methods, unless, multiple when clauses, context."""
import json
import random

USERS = [f"u{i}" for i in range(6)]
GROUPS = [f"g{i}" for i in range(6)]
TAGS = ["t0", "t1", "t2", "t3", "prod-x", "x*y"]
# Cedar pattern literals as they appear in policy text ("x\*y" matches the literal star)
PATTERNS = ['"u*"', '"*1"', '"u*1"', '"*"', '"prod-*"', '"x\\*y"', '"*-*"', '"u0"', '""', '"n*s*1"', '"**"', '"t*t"']


def q(s):
    return json.dumps(s)


# groups only the image's static entities know (static mode)
SGROUPS = [f"s{i}" for i in range(4)]


class Gen:
    def __init__(self, seed, static=False):
        self.r = random.Random(seed)
        self.static = static
        self.groups = GROUPS + SGROUPS if static else GROUPS

    def pick(self, xs):
        return self.r.choice(xs)

    def long_e(self, d=0):
        r = self.r
        opts = [lambda: str(r.randint(-5, 50)), lambda: "principal.age", lambda: "context.x", lambda: "resource.size",
                lambda: "principal.info.a", lambda: "9223372036854775807", lambda: "-9223372036854775808"]
        if d < 2:
            opts += [lambda: f"({self.long_e(d + 1)} {r.choice(['+', '-', '*'])} {self.long_e(d + 1)})",
                     lambda: f"-{self.long_e(d + 1)}",
                     lambda: f"(if {self.bool_e(d + 1)} then {self.long_e(d + 1)} else {self.long_e(d + 1)})"]
        return r.choice(opts)()

    def str_e(self, d=0):
        r = self.r
        return r.choice([lambda: q(r.choice(USERS + TAGS + ["", "ns1"])), lambda: "principal.name",
                         lambda: "resource.name", lambda: "resource.namespace", lambda: "principal.info.b",
                         lambda: "context.s"])()

    def ent_e(self, d=0):
        r = self.r
        return r.choice([lambda: "principal", lambda: "resource", lambda: "resource.owner", lambda: "action",
                         lambda: f'k8s::Group::{q(r.choice(self.groups))}', lambda: f'k8s::User::{q(r.choice(USERS))}'])()

    def set_e(self, d=0):
        r = self.r
        return r.choice([lambda: "principal.tags", lambda: "resource.labels", lambda: "context.list",
                         lambda: "[" + ", ".join(q(x) for x in r.sample(TAGS, r.randint(0, 3))) + "]",
                         lambda: f"[{self.str_e(d + 1)}, {q(r.choice(TAGS))}]",
                         lambda: f"[{self.long_e(d + 1)}, 3]",
                         lambda: "[" + ", ".join(f"k8s::Group::{q(g)}" for g in r.sample(self.groups, 2)) + "]",
                         lambda: f'[{{"key": {q(r.choice(["k0", "k1"]))}, "value": {self.str_e(d + 1)}}}]',
                         lambda: "principal.info.c"])()

    def any_e(self, d=0):
        return "(" + self.r.choice([self.long_e, self.str_e, self.ent_e, self.set_e, self.bool_e])(d + 1) + ")"

    def bool_e(self, d=0):
        r = self.r
        leaves = [
            lambda: "principal.active", lambda: "context.flag", lambda: r.choice(["true", "false"]),
            lambda: f"{r.choice(['principal', 'resource', 'context', 'principal.info'])} has {r.choice(['name', 'namespace', 'age', 'tags', 'a', 'x', 'info', 'owner'])}",
            lambda: f"{self.ent_e(d)} in k8s::Group::{q(r.choice(self.groups))}",
            lambda: f"{self.ent_e(d)} in {self.set_e(d)}",
            lambda: f"{self.ent_e(d)} is {r.choice(['k8s::User', 'k8s::Group', 'k8s::Resource'])}",
            lambda: f"principal is k8s::User in k8s::Group::{q(r.choice(self.groups))}",
            lambda: f"{self.long_e(d)} {r.choice(['<', '<=', '>', '>='])} {self.long_e(d)}",
            lambda: f"{self.str_e(d)} {r.choice(['==', '!='])} {self.str_e(d)}",
            lambda: f"{self.any_e(d)} {r.choice(['==', '!='])} {self.any_e(d)}",
            lambda: f"{self.set_e(d)} == {self.set_e(d)}",
            lambda: f"{self.str_e(d)} like {r.choice(PATTERNS)}",
            lambda: f"{self.set_e(d)}.contains({self.any_e(d)})",
            lambda: f"{self.set_e(d)}.{r.choice(['containsAll', 'containsAny'])}({self.set_e(d)})",
            lambda: f"{self.set_e(d)}.isEmpty()",
            lambda: f'resource.ip.{r.choice(["isIpv4", "isIpv6", "isLoopback", "isMulticast"])}()',
            lambda: f'resource.ip.isInRange(ip({q(r.choice(["10.0.0.0/8", "127.0.0.0/8", "::1/128", "192.168.1.0/24"]))}))',
            lambda: f'resource.score.{r.choice(["lessThan", "lessThanOrEqual", "greaterThan", "greaterThanOrEqual"])}(decimal({q(r.choice(["1.5", "-2.25", "0.0001"]))}))',
            lambda: f'resource.labels.contains({{"key": {q(r.choice(["k0", "k1"]))}, "value": {self.str_e(d)}}})',
            lambda: f'{self.any_e(d)}',  # possibly non-bool -> type errors
        ]
        if d < 3:
            leaves += [lambda: f"({self.bool_e(d + 1)} && {self.bool_e(d + 1)})",
                       lambda: f"({self.bool_e(d + 1)} || {self.bool_e(d + 1)})",
                       lambda: f"!{self.bool_e(d + 1)}",
                       lambda: f"(if {self.bool_e(d + 1)} then {self.bool_e(d + 1)} else {self.bool_e(d + 1)})"]
        return r.choice(leaves)()

    def scope(self, var):
        r = self.r
        t = r.random()
        if t < 0.4:
            return var
        if var == "action":
            if t < 0.7:
                return "action in [" + ", ".join(f"k8s::Action::{q(v)}" for v in r.sample(["get", "list", "watch", "create"], 2)) + "]"
            return f'action == k8s::Action::{q(r.choice(["get", "list"]))}'
        if t < 0.55:
            return f"{var} is {r.choice(['k8s::User', 'k8s::Resource', 'k8s::Group'])}"
        if t < 0.7:
            return f"{var} in k8s::Group::{q(r.choice(self.groups))}"
        if t < 0.85:
            return f"{var} is k8s::User in k8s::Group::{q(r.choice(self.groups))}"
        if var == "principal":
            return f"principal == k8s::User::{q(r.choice(USERS))}"
        return f"resource == k8s::Resource::{q('r' + str(r.randint(0, 3)))}"

    def policy(self):
        r = self.r
        eff = "forbid" if r.random() < 0.3 else "permit"
        conds = []
        for _ in range(r.choice([0, 1, 1, 2, 3])):
            conds.append(f"{r.choice(['when', 'when', 'unless'])} {{ {self.bool_e()} }}")
        ann = "@id(\"x\")\n" if r.random() < 0.2 else ""
        return f"{ann}{eff} ({self.scope('principal')}, {self.scope('action')}, {self.scope('resource')})\n" + "\n".join(conds) + ";"

    def policies(self, n):
        return "\n".join(self.policy() for _ in range(n))

    # ---- policies the device compiler lowers to predicate atoms (conjunction/disjunction chains
    # over request attributes), incl. the label-selector template shape
    def sel_tmpl(self):
        r = self.r
        key = q(r.choice(["k0", "k1", "owner"]))
        v = lambda: r.choice([q(r.choice(USERS + TAGS)), "principal.name", "principal.nick"])
        t = r.random()
        if t < 0.4:
            vals = ", ".join(v() for _ in range(r.randint(0, 2)))
            return f'{{"key": {key}, "operator": "in", "values": [{vals}]}}'
        if t < 0.7:
            return f'{{"key": {key}, "value": {v()}}}'
        return f'{{"operator": {q(r.choice(["in", "notin"]))}, "key": {key}, "values": [{v()}]}}'

    def atom_e(self):
        r = self.r
        return r.choice([
            lambda: "resource has sel", lambda: "principal has nick", lambda: "principal.active",
            lambda: f'resource.namespace == {q(r.choice(["ns1", "ns2", "u0"]))}',
            lambda: f'resource.namespace != {q(r.choice(["ns1", "ns2"]))}',
            lambda: f"resource.name like {r.choice(PATTERNS)}",
            lambda: f"principal.age {r.choice(['<', '<=', '>', '>='])} {r.randint(-5, 50)}",
            lambda: "resource.name == principal.name",
            lambda: f'{q(r.choice(USERS))} == principal.name',
            lambda: f"principal in k8s::Group::{q(r.choice(self.groups))}",
            lambda: f"principal is {r.choice(['k8s::User', 'k8s::Group'])}",
            lambda: "[" + ", ".join(q(x) for x in r.sample(TAGS + USERS, 3)) + "].contains(resource.name)",
            lambda: f"principal.tags.contains({q(r.choice(TAGS))})",
            lambda: "resource.sel.containsAny([" + ", ".join(self.sel_tmpl() for _ in range(r.randint(1, 3))) + "])",
            lambda: f"resource.sel.contains({self.sel_tmpl()})",
            lambda: f"!resource.sel.containsAny([{self.sel_tmpl()}])",
            # nested attribute paths (host-resolved hot paths), incl. through an entity reference
            lambda: f"principal.info.a {r.choice(['<', '>=', '=='])} {r.randint(-3, 9)}",
            lambda: f'principal.info.b == {q(r.choice(TAGS))}',
            lambda: "principal.info has c", lambda: "principal has info && principal.info has c",
            lambda: f'resource.owner.name == {q(r.choice(USERS))}',
            lambda: "resource has owner && resource.owner has name",
            lambda: f'principal.info.c.contains({q(r.choice(TAGS))})',
            lambda: f"context.x {r.choice(['<', '>'])} {r.randint(0, 40)}",
            lambda: "context.flag", lambda: "context has s && context.s == principal.name",
            # entity set membership, is-in, var == literal, constants
            lambda: "resource in [" + ", ".join(f"k8s::Group::{q(g)}" for g in r.sample(self.groups, 2)) + "]",
            lambda: f"principal in [k8s::Group::{q(r.choice(self.groups))}, k8s::User::{q(r.choice(USERS))}]",
            lambda: f"principal is k8s::User in k8s::Group::{q(r.choice(self.groups))}",
            lambda: f'resource == k8s::Resource::{q("r" + str(r.randint(0, 3)))}',
            lambda: f'principal == k8s::User::{q(r.choice(USERS))}',
            lambda: r.choice(["true", "false"]),
        ])()

    def atom_tree(self, d=0):
        r = self.r
        t = r.random()
        if d >= 2 or t < 0.45:
            return self.atom_e()
        if t < 0.65:
            return f"({self.atom_tree(d + 1)} && {self.atom_tree(d + 1)})"
        if t < 0.85:
            return f"({self.atom_tree(d + 1)} || {self.atom_tree(d + 1)})"
        if t < 0.93:
            return f"!({self.atom_tree(d + 1)})"
        return f"(if {self.atom_tree(d + 1)} then {self.atom_tree(d + 1)} else {self.atom_tree(d + 1)})"

    def atomic_policy(self):
        r = self.r
        eff = "forbid" if r.random() < 0.25 else "permit"
        conds = []
        for _ in range(r.choice([0, 1, 1, 2])):
            if r.random() < 0.5:
                op = " || " if r.random() < 0.3 else " && "
                body = op.join(self.atom_e() for _ in range(r.randint(1, 4)))
            else:
                body = self.atom_tree()
            conds.append(f"{r.choice(['when', 'when', 'unless'])} {{ {body} }}")
        return f"{eff} ({self.scope('principal')}, {self.scope('action')}, {self.scope('resource')})\n" + "\n".join(conds) + ";"

    def atomic_policies(self, n):
        return "\n".join(self.atomic_policy() for _ in range(n))

    def sel_value(self):
        r = self.r
        if r.random() < 0.05:
            return "not-a-set"
        out = []
        for _ in range(r.randint(0, 3)):
            key = r.choice(["k0", "k1", "owner"])
            t = r.random()
            if t < 0.5:
                out.append({"key": key, "operator": "in", "values": r.sample(USERS[:3] + TAGS[:2], r.randint(0, 2))})
            elif t < 0.75:
                out.append({"key": key, "value": r.choice(USERS[:3] + TAGS[:2])})
            elif t < 0.85:
                out.append({"key": key, "operator": "in", "values": [r.choice(USERS[:3])], "extra": 1})
            elif t < 0.95:
                out.append(r.choice(USERS))
            else:
                out.append({"key": key, "operator": "in", "values": [r.choice(USERS[:3]), r.choice(USERS[:3])]})
        return out

    def value_attrs_user(self):
        r = self.r
        a = {"name": r.choice(USERS)}
        if r.random() < 0.85:
            a["age"] = r.choice([r.randint(0, 60), 2 ** 40, -(2 ** 35)])
        if r.random() < 0.8:
            a["tags"] = r.sample(TAGS, r.randint(0, 4))
        if r.random() < 0.8:
            info = {"a": r.randint(-3, 9), "b": r.choice(TAGS)}
            if r.random() < 0.7:
                info["c"] = r.sample(TAGS, r.randint(0, 3))
            a["info"] = info
        if r.random() < 0.8:
            a["active"] = r.random() < 0.5
        if r.random() < 0.6:
            a["nick"] = r.choice(USERS[:3] + TAGS[:2])
        return a

    def static_entities(self):
        """A static hierarchy for the image (cg_compiler_set_entities): groups g*/s* with parents
        among later groups (a DAG, sometimes a cycle), static-only users u4/u5 in groups, and a
        static resource r3 with attributes."""
        r = self.r
        out = []
        allg = GROUPS + SGROUPS
        for i, g in enumerate(allg):
            later = allg[i + 1:]
            par = r.sample(later, min(len(later), r.choice([0, 1, 1, 2]))) if later else []
            if r.random() < 0.05:
                par.append(r.choice(allg[:i + 1]))  # a cycle now and then
            out.append({"uid": {"type": "k8s::Group", "id": g}, "attrs": {"name": g, "level": i},
                        "parents": [{"type": "k8s::Group", "id": p} for p in par]})
        for u in ("u4", "u5"):
            out.append({"uid": {"type": "k8s::User", "id": u}, "attrs": self.value_attrs_user(),
                        "parents": [{"type": "k8s::Group", "id": g} for g in r.sample(allg, 2)]})
        out.append({"uid": {"type": "k8s::Resource", "id": "r3"}, "attrs": {"name": "r3", "size": 7, "namespace": "ns1"},
                    "parents": [{"type": "k8s::Group", "id": r.choice(SGROUPS)}]})
        return out

    def item(self):
        r = self.r
        ents = []
        groups = r.sample(GROUPS, r.randint(0, 3))
        puid = {"type": "k8s::User", "id": r.choice(USERS)}
        if self.static and puid["id"] in ("u4", "u5") and r.random() < 0.7:
            pass  # the principal is only a static entity
        else:
            ents.append({"uid": puid, "attrs": self.value_attrs_user(),
                         "parents": [{"type": "k8s::Group", "id": g} for g in groups]})
        # group hierarchy g_i -> g_{i+1} (static mode: mostly parentless group entities, as the SAR
        # path builds them, which the static hierarchy then re-parents; sometimes a request edge of
        # its own on a static group)
        for g in GROUPS:
            if r.random() < 0.7:
                i = int(g[1:])
                chance = 0.1 if self.static else 0.6
                par = [{"type": "k8s::Group", "id": f"g{i + 1}"}] if i + 1 < len(GROUPS) and r.random() < chance else []
                ents.append({"uid": {"type": "k8s::Group", "id": g}, "attrs": {"name": g}, "parents": par})
        ruid = {"type": "k8s::Resource", "id": f"r{r.randint(0, 3)}"}
        ra = {"name": r.choice(TAGS + USERS), "size": r.randint(-10, 100)}
        if r.random() < 0.6:
            ra["namespace"] = r.choice(["ns1", "ns2", "u0"])
        if r.random() < 0.7:
            ra["owner"] = {"__entity": {"type": "k8s::User", "id": r.choice(USERS)}}
        if r.random() < 0.7:
            ra["labels"] = [{"key": r.choice(["k0", "k1"]), "value": r.choice(USERS + TAGS)} for _ in range(r.randint(0, 3))]
        if r.random() < 0.7:
            ra["ip"] = {"__extn": {"fn": "ip", "arg": r.choice(["10.1.2.3", "127.0.0.1", "::1", "192.168.1.7/24", "224.0.0.1", "ff02::1"])}}
        if r.random() < 0.7:
            ra["score"] = {"__extn": {"fn": "decimal", "arg": r.choice(["1.5", "-3.0", "0.0001", "12.3456"])}}
        if r.random() < 0.75:
            ra["sel"] = self.sel_value()
        if r.random() < 0.9:
            ents.append({"uid": ruid, "attrs": ra, "parents": [{"type": "k8s::Group", "id": r.choice(self.groups)}] if r.random() < 0.3 else []})
        act = {"type": "k8s::Action", "id": r.choice(["get", "list", "watch", "create"])}
        ctx = {}
        if r.random() < 0.8:
            ctx["x"] = r.randint(-5, 50)
        if r.random() < 0.8:
            ctx["flag"] = r.random() < 0.5
        if r.random() < 0.6:
            ctx["list"] = [r.randint(0, 5) for _ in range(r.randint(0, 3))]
        if r.random() < 0.5:
            ctx["s"] = r.choice(USERS)
        return ents, {"principal": puid, "action": act, "resource": ruid, "context": ctx}

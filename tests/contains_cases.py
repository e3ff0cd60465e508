"""Set-membership shapes the scope index files under element hashes (image.h BT_CKEY): contains
of primitives and of constant record templates, guarded and unguarded, on sets holding records
with other keys, nested values, large longs, entities, and on values that are no set (errors)."""
import random

POLICIES = r'''
forbid (principal, action, resource is k8s::Resource) when { resource has data && resource.data.contains({"key": "k1", "value": "v1"}) };
forbid (principal, action, resource is k8s::Resource) when { resource has data && resource.data.contains({"key": "k2", "value": "v9"}) };
permit (principal, action, resource) when { resource.tags.contains("red") };
permit (principal, action == k8s::Action::"get", resource) when { context.nums.contains(5) };
permit (principal, action, resource) when { context has nums && context.nums.contains(9223372036854775807) };
permit (principal, action, resource) when { context has nums && context.nums.contains(-1) && context.n == 3 };
forbid (principal, action, resource) when { context has ents && context.ents.contains(k8s::User::"alice") };
forbid (principal, action, resource) when { context has recs && context.recs.contains({"a": 1, "b": true}) };
permit (principal, action, resource) when { context has recs && context.recs.contains({"who": k8s::User::"bob"}) };
permit (principal, action, resource) when { context has tags && context.tags.contains("x") || context.n == 1 };
permit (principal is k8s::User, action, resource) when { context has tags && context.tags.contains(true) };
forbid (principal, action, resource) unless { resource has data && resource.data.contains({"key": "owner", "value": "alice"}) };
'''

_DATA = [{"key": "k1", "value": "v1"}, {"key": "k2", "value": "v9"}, {"key": "k1", "value": "v2"},
         {"key": "k1", "value": "v1", "x": 1}, {"key": "owner", "value": "alice"}, {"key": "k1"},
         {"key": "k1", "value": {"nested": 1}}]
_TAGS = ["red", "blue", "x", True, 5, "RED"]
_NUMS = [5, 6, -1, 9223372036854775807, 1 << 40, -9223372036854775808]
_RECS = [{"a": 1, "b": True}, {"a": 1}, {"a": 1, "b": False}, {"who": {"__entity": {"type": "k8s::User", "id": "bob"}}},
         {"who": "bob"}, {"a": 1, "b": True, "c": 0}]


def _pick(r, pool, k):
    return [r.choice(pool) for _ in range(r.randint(0, k))]


def items(n=400, seed=0):
    r = random.Random(seed)
    out = []
    for k in range(n):
        rattrs = {}
        x = r.random()
        if x < 0.6:
            rattrs["data"] = _pick(r, _DATA, 4)
        elif x < 0.7:
            rattrs["data"] = {"key": "k1", "value": "v1"}  # a record, not a set: contains raises
        x = r.random()
        if x < 0.7:
            rattrs["tags"] = _pick(r, _TAGS, 4)
        elif x < 0.8:
            rattrs["tags"] = "red"
        ctx = {"n": r.randint(0, 4)}
        if r.random() < 0.7:
            ctx["nums"] = _pick(r, _NUMS, 4)
        elif r.random() < 0.5:
            ctx["nums"] = 5
        if r.random() < 0.5:
            ctx["ents"] = [{"__entity": {"type": "k8s::User", "id": r.choice(["alice", "bob"])}} for _ in range(r.randint(0, 2))]
        if r.random() < 0.6:
            ctx["recs"] = _pick(r, _RECS, 3)
        if r.random() < 0.4:
            ctx["tags"] = _pick(r, _TAGS, 3)
        ents = [{"uid": {"type": "k8s::Resource", "id": "r"}, "attrs": rattrs, "parents": []},
                {"uid": {"type": "k8s::User", "id": "u"}, "attrs": {}, "parents": []}]
        req = {"principal": {"type": "k8s::User", "id": "u"},
               "action": {"type": "k8s::Action", "id": r.choice(["get", "list"])},
               "resource": {"type": "k8s::Resource", "id": "r" if r.random() < 0.9 else "other"}, "context": ctx}
        out.append((ents, req))
    return out

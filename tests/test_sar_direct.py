"""Direct SubjectAccessReview encoder (sar.cpp encode_sar_direct: views into the body, no JSON /
Attributes / HVal trees) against the general path (json_parse -> attributes_from_sar ->
record_to_cedar -> encode_request), word for word, through cg_encode_sar_check. Host only.

The general path is itself pinned to the reference's entity construction
(authorizer_test.go:31-460 vectors in test_encoder / test_sar); this test pins the direct path to
it, including the SAR shapes the direct path hands back (escapes, numbers, merged extra keys)."""
import ctypes
import json
import os
import random

import cedargpu
from cedargpu import synth
from cedargpu._lib import lib
from conftest import GOLDEN

CORPUS = json.load(open(os.path.join(GOLDEN, "reference_corpus.json")))


def check(image: bytes, sars_text: str):
    b = sars_text.encode("utf-8")
    n, nd, nm = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    first = ctypes.c_int64()
    rc = lib.cg_encode_sar_check(image, len(image), b, len(b), ctypes.byref(n), ctypes.byref(nd), ctypes.byref(nm),
                                 ctypes.byref(first))
    assert rc == 0
    return n.value, nd.value, nm.value, first.value


def _abac_image(pop):
    return cedargpu.build_image([cedargpu.MemoryStore("c3.cedar", synth.abac_policies(600, seed=3, pop=pop))])


def _demo_image():
    text = "\n".join(v for k, v in sorted(CORPUS["demo"].items()))
    files = dict(CORPUS["converter"])
    return cedargpu.build_image([cedargpu.DirectoryStore(files), cedargpu.MemoryStore("demo.cedar", text)])


def test_synthetic_sars_take_the_direct_path_and_match():
    pop = synth.Population(seed=7, n_users=4000, n_groups=300)
    sars = synth.random_sars(4000, seed=11, pop=pop)
    for image in (_abac_image(pop), _demo_image()):
        n, nd, nm, first = check(image, json.dumps(sars))
        assert n == len(sars)
        assert nm == 0, sars[first]
        assert nd == n  # plain bodies never need the general path


def test_static_hierarchy_image_encodes_alike():
    """An image with a static group DAG: both paths merge the hierarchy into the request the same
    way (closure rows, key-entity-first ancestor order)."""
    pop = synth.Population(seed=8, n_users=3000, n_groups=400, dag_depth=12)
    image = cedargpu.build_image([cedargpu.MemoryStore("c3.cedar", synth.abac_policies(600, seed=3, pop=pop))],
                                 entities=pop.static_entities())
    sars = synth.random_sars(3000, seed=12, pop=pop)
    n, nd, nm, first = check(image, json.dumps(sars))
    assert n == len(sars) and nd == n
    assert nm == 0, sars[first]


def _variants(rng: random.Random):
    """SubjectAccessReview bodies around every branch of GetAuthorizerAttributes and
    RecordToCedarResource, plus shapes the direct path must hand to the general path."""
    users = ["alice", "Bob", "system:node:n1", "system:node:a:b", "system:serviceaccount:ns1:sa1",
             "system:serviceaccount:a:b:c", "system:masters", "system:authorizer:cedar-authorizer", "", "ü-ser",
             "system:serviceaccount:x", "system:nodes"]
    groups = [[], ["g1"], ["g1", "g1", "g2"], ["system:authenticated", "dev"], [1, "g3"], {"a": 1}]
    verbs = ["get", "list", "watch", "create", "impersonate", "delete", ""]
    resources = ["pods", "policies", "roles", "serviceaccounts", "uids", "users", "groups", "userextras", "secrets", ""]
    api_groups = ["", "apps", "cedar.k8s.aws", "rbac.authorization.k8s.io"]
    out = []
    for i in range(3000):
        spec = {}
        if rng.random() < 0.95:
            spec["user"] = rng.choice(users) if rng.random() < 0.97 else True
        if rng.random() < 0.9:
            spec["uid"] = rng.choice(["uid-1", "", "alice", "g1", "system:node:n1"])
        if rng.random() < 0.8:
            spec["groups"] = rng.choice(groups)
        r = rng.random()
        if r < 0.1:
            spec["extra"] = {"Scopes": ["a", "b", "a"], "team": ["x"], "N": 3}
        elif r < 0.15:
            spec["extra"] = {"k": "notalist", "K2": []}
        elif r < 0.17:
            spec["extra"] = ["bad"]
        ra = {}
        for k, vals in (("verb", verbs), ("resource", resources), ("group", api_groups),
                        ("namespace", ["", "default", "kube-system"]), ("version", ["v1", ""]),
                        ("name", ["", "n", "system:node:w", "system:node:a:b"]),
                        ("subresource", ["", "status", "scale"])):
            if rng.random() < 0.85:
                ra[k] = rng.choice(vals)
        if rng.random() < 0.2:
            ra["labelSelector"] = {"requirements": [
                {"key": rng.choice(["app", "bad key", "x.io/y", "-bad", "a" * 70]),
                 "operator": rng.choice(["In", "NotIn", "Exists", "DoesNotExist", "Gt"]),
                 "values": rng.choice([[], ["v"], ["v", "w", "v"], ["bad value!"], "x"])}
                for _ in range(rng.randint(0, 3))] + ([7] if rng.random() < 0.2 else [])}
        if rng.random() < 0.2:
            ra["fieldSelector"] = {"requirements": [
                {"key": rng.choice(["metadata.name", "spec.nodeName"]),
                 "operator": rng.choice(["In", "NotIn", "Exists"]),
                 "values": rng.choice([[], ["a"], ["a", "b"]])} for _ in range(rng.randint(0, 3))]}
        if rng.random() < 0.85:
            spec["resourceAttributes"] = ra if rng.random() < 0.97 else "notanobject"
        if rng.random() < 0.15:
            spec["nonResourceAttributes"] = {"path": rng.choice(["/healthz", "/api", ""]),
                                             "verb": rng.choice(["get", "post"])}
        body = {"apiVersion": "authorization.k8s.io/v1", "kind": "SubjectAccessReview", "spec": spec}
        text = json.dumps(body, ensure_ascii=rng.random() < 0.5, indent=rng.choice([None, None, 1]))
        r = rng.random()
        if r < 0.03:
            text = text.replace('"spec"', '"spec": {"user": "dup"}, "spec"', 1)  # duplicate key: first wins
        elif r < 0.05:
            text = text.replace('"uid"', '"uid": "u\\/x", "uid"', 1)  # escape: general path
        elif r < 0.07:
            text = text.replace('"kind"', '"n": 1.5, "kind"', 1)  # number: general path
        out.append(text)
    return out


def test_variant_sars_match_general_path():
    pop = synth.Population(seed=7, n_users=500, n_groups=40)
    rng = random.Random(5)
    texts = _variants(rng)
    payload = "[" + ",".join(texts) + "]"
    for image in (_abac_image(pop), _demo_image()):
        n, nd, nm, first = check(image, payload)
        assert n == len(texts)
        assert nm == 0, texts[first]
        assert nd > 0.5 * n, (nd, n)  # numbers and escapes in the variants go to the general path


def test_malformed_bodies_are_left_to_the_general_path():
    image = _demo_image()
    for bad in ['{"spec": {"user": "a",}}', '{"spec": [1]}', '{"kind": "x"}', '[{"spec": {}}]', '{"spec": {"user": tru}}']:
        n, nd, nm, _ = check(image, "[" + bad + "]")
        assert (n, nd, nm) == (1, 0, 0), bad


def test_ancestor_count_limits_of_the_row_format():
    """The request row packs an entity's ancestor count into 16 bits (image.h AN_COUNT: 65,535)
    and its key-ancestor count into 15 (AN_KEYS: 32,767; cedargpu.h documents both): a user in
    65,535 groups encodes, one in 65,536 is refused by the encoder (an error for that request,
    never a truncated list)."""
    img = _demo_image()

    def sar(n_groups):
        s = synth.make_sar("big-user", "u1", [f"g{k}" for k in range(n_groups)], "get", ns="default", resource="pods")
        return json.dumps([s])

    b = sar(65535).encode()
    n, nd, nm, first = (ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_int64())
    assert lib.cg_encode_sar_check(img, len(img), b, len(b), ctypes.byref(n), ctypes.byref(nd), ctypes.byref(nm),
                                   ctypes.byref(first)) == 0
    assert n.value == 1 and nm.value == 0
    b = sar(65536).encode()
    rc = lib.cg_encode_sar_check(img, len(img), b, len(b), ctypes.byref(n), ctypes.byref(nd), ctypes.byref(nm),
                                 ctypes.byref(first))
    assert rc != 0


def test_closure_cache_matches_the_hierarchy_walk():
    """The encoder's per-thread ancestor-record cache (encode_impl.h ClosureCache: static closure
    rows, unions of parents' closures) against the general hierarchy walk, word for word, on random
    EntityMaps over random static hierarchies: request edges on static groups, static-only
    principals, cycles, re-parented static targets (which must take the walk). Host only."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from randgen import Gen
    for seed in range(6):
        g = Gen(900 + seed, static=True)
        ents = g.static_entities()
        image = cedargpu.build_image([cedargpu.MemoryStore("p.cedar", synth.abac_policies(200, seed=seed))], entities=ents)
        items = []
        for _ in range(300):
            e, r = g.item()
            items.append({"entities": e, "request": r})
        b = json.dumps(items).encode()
        n, nm, first = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_int64()
        assert lib.cg_encode_items_check(image, len(image), b, len(b), ctypes.byref(n), ctypes.byref(nm),
                                         ctypes.byref(first)) == 0
        assert n.value == len(items)
        assert nm.value == 0, items[first.value]


def _split(text: str, threads: int):
    b = text.encode("utf-8")
    n, same = ctypes.c_int64(), ctypes.c_int()
    assert lib.cg_json_split_check(b, len(b), threads, ctypes.byref(n), ctypes.byref(same)) == 0
    return n.value, same.value


def test_parallel_array_split_matches_serial():
    """The bulk paths split a large JSON array on several threads (capi.cpp split_array_regions:
    quote parity per region, prefix sums, separators at the array's level). Against the serial
    scan, element for element: strings holding brackets, commas, escaped quotes and backslash runs
    that straddle region boundaries, nested values, scalars, whitespace, malformed arrays."""
    r = random.Random(5)
    pieces = ['"a,b"', '"[{"', '"}]"', '"x\\\\"', '"q\\"[,"', '"\\\\\\"}"', '{"k": [1, {"z": "]"}], "v": "\\\\"}',
              '[1, 2, [3]]', '17', 'true', 'null', '{"s": "a\\\\\\\\"}', '{ }', '[ ]', '"\\u005b"']
    for _ in range(300):
        els = [r.choice(pieces) for _ in range(r.randint(0, 40))]
        sep = r.choice([",", ", ", " ,\n", ","])
        text = r.choice(["", " ", "\n"]) + "[" + r.choice(["", " "]) + sep.join(els) + r.choice(["", " "]) + "]"
        for threads in (2, 3, 7, 16, 61):
            n, same = _split(text, threads)
            assert same == 1, (text, threads)
            assert n == len(els)
    for bad in ["[1,,2]", "[,1]", "[1", '["a]', "{}", "[1]]", '[1, "\\"]']:
        for threads in (2, 5):
            n, same = _split(bad, threads)
            assert same == 1, (bad, threads)
    sars = synth.random_sars(3000, seed=9, pop=synth.Population(seed=9, n_users=500, n_groups=40))
    text = json.dumps(sars)
    for threads in (2, 8, 16, 64):
        n, same = _split(text, threads)
        assert same == 1 and n == len(sars)

"""CPU-only checks of the native library: it loads, exports every declared symbol, compiles the
reference corpus, and its C++ SubjectAccessReview model matches the reference vectors / oracle."""
import json
import os
import re

import pytest

import cedar_oracle as co
import k8s_model as km
from conftest import GOLDEN, ROOT
from helpers import attrs_from, cxx_sar_to_cedar, norm_entities, sar_from_attrs
from randgen import Gen

import cedargpu
from cedargpu import synth

V = json.load(open(os.path.join(GOLDEN, "reference_vectors.json")))
CORPUS = json.load(open(os.path.join(GOLDEN, "reference_corpus.json")))


def test_exports_every_declared_symbol():
    hdr = open(os.path.join(ROOT, "include", "cedargpu.h")).read()
    declared = set(re.findall(r"\b(cg_[a-z_0-9]+)\s*\(", hdr))
    assert len(declared) >= 30
    for name in declared:
        assert hasattr(cedargpu.lib, name), name
    assert declared == set(cedargpu._lib.EXPORTED)


def test_metrics_layout_and_buckets():
    """cg_queue_metrics (the reference's request_total / request_duration_seconds, metrics.go:27-47):
    the binding's struct matches the header's, and the latency buckets hold the reference's."""
    import ctypes
    hdr = open(os.path.join(ROOT, "include", "cedargpu.h")).read()
    nb = int(re.search(r"#define CG_LAT_BOUNDS (\d+)", hdr).group(1))
    nz = int(re.search(r"#define CG_BATCH_BUCKETS (\d+)", hdr).group(1))
    assert (nb, nz) == (cedargpu.store.LAT_BOUNDS, cedargpu.store.BATCH_BUCKETS)
    body = re.search(r"typedef struct cg_queue_metrics \{(.*?)\} cg_queue_metrics;", hdr, re.S).group(1)
    words = 0
    for m in re.finditer(r"uint64_t (\w+)((?:\[[^\]]+\])*);", body):
        n = 1
        for dim in re.findall(r"\[([^\]]+)\]", m.group(2)):
            n *= eval(dim.replace("CG_LAT_BOUNDS", str(nb)).replace("CG_BATCH_BUCKETS", str(nz)))
        words += n
    assert ctypes.sizeof(cedargpu.store.QueueMetrics) == 8 * words
    n = ctypes.c_uint32()
    bp = cedargpu.lib.cg_metrics_latency_bounds(ctypes.byref(n))
    bounds = [bp[i] for i in range(n.value)]
    assert n.value == nb and bounds == sorted(bounds)
    for sec in (0.25, 0.5, 0.7, 1, 1.5, 3, 5, 10):
        assert round(sec * 1e9) in bounds
    assert cedargpu.lib.cg_queue_metrics_get(None, None, 0) != 0


def test_version():
    assert b"gfx950" in cedargpu.lib.cg_version()


@pytest.mark.parametrize("name", sorted(CORPUS["converter"]) + sorted(CORPUS["demo"]))
def test_corpus_compiles(name):
    src = CORPUS["converter"].get(name) or CORPUS["demo"][name]
    img = cedargpu.build_image([cedargpu.MemoryStore(name, src)])
    import ctypes
    n, t, e = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint64()
    assert cedargpu.lib.cg_image_info(img, len(img), ctypes.byref(n), ctypes.byref(t), ctypes.byref(e)) == 0
    assert n.value == len(co.parse_policies(src, name))
    assert t.value == 1


def test_parse_error_is_reported():
    with pytest.raises(cedargpu.CompileError):
        cedargpu.build_image([cedargpu.MemoryStore("bad", "permit(principal, action, resource) when { 1 + };")])
    with pytest.raises(cedargpu.CompileError):
        cedargpu.build_image([cedargpu.MemoryStore("bad", "allow(principal, action, resource);")])


def test_tiers_and_id_conventions_compile():
    stores = [cedargpu.DirectoryStore({"a.cedar": "permit(principal, action, resource);", "skip.txt": "x"}),
              cedargpu.CRDStore([("pol", "u-1", "forbid(principal, action, resource);")]),
              cedargpu.AVPStore([("avp1", "permit(principal, action, resource);")]),
              cedargpu.ALLOW_ALL_ADMISSION]
    img = cedargpu.build_image(stores)
    import ctypes
    n, t = ctypes.c_uint32(), ctypes.c_uint32()
    cedargpu.lib.cg_image_info(img, len(img), ctypes.byref(n), ctypes.byref(t), None)
    assert (n.value, t.value) == (4, 4)


@pytest.mark.parametrize("case", [c for c in V["record_to_cedar"] if not c["attributes"].get("label_selector")],
                         ids=lambda c: c["name"])
def test_cxx_sar_model_matches_reference_vectors(case):
    """C++ RecordToCedarResource == authorizer_test.go:31-460 (selector-free cases: those
    selectors use operator "=", which a SubjectAccessReview cannot express)."""
    got = cxx_sar_to_cedar(sar_from_attrs(case["attributes"]))
    assert norm_entities(got["entities"]) == norm_entities(case["want_entities"])
    assert got["request"] == case["want_request"]


def test_cxx_sar_model_matches_oracle_on_synthetic_sars():
    sars = synth.random_sars(3000, seed=5, pop=synth.Population(seed=3, n_users=2000, n_groups=300))
    sars.append(synth.make_sar("a", "u", ["g"], "list", ns="d", resource="pods", version="v1", label_selector=[
        {"key": "owner", "operator": "In", "values": ["a", "b"]}, {"key": "bad key", "operator": "In", "values": ["x"]},
        {"key": "e", "operator": "Exists"}, {"key": "x", "operator": "Exists", "values": ["v"]}]))
    sars.append({"spec": {"user": "u", "uid": "1", "resourceAttributes": {"verb": "list", "resource": "pods", "version": "v1",
                 "fieldSelector": {"requirements": [{"key": "a", "operator": "In", "values": ["1"]},
                                                    {"key": "b", "operator": "NotIn", "values": ["2"]},
                                                    {"key": "c", "operator": "Exists"}]}}}})
    sars.append(synth.make_sar("system:authorizer:cedar-authorizer", "", [], "get", group="cedar.k8s.aws",
                               resource="policies"))
    sars.append(synth.make_sar("system:kube-scheduler", "", [], "get", resource="pods"))
    n_fast = 0
    for sar in sars:
        got = cxx_sar_to_cedar(sar)
        a = km.attributes_from_sar(sar)
        if "fast" in got:
            n_fast += 1
            dec, reason = km.authorize([], a)
            assert (got["fast"], got["reason"]) == (dec, reason)
            continue
        em, req = km.record_to_cedar_resource(a)
        assert norm_entities(got["entities"]) == norm_entities(co.entities_to_json(em)), sar
        assert got["request"] == co.request_to_json(req)
    assert n_fast >= 2


@pytest.mark.parametrize("seed", range(8))
def test_atomic_generator_lowers_every_policy_to_atoms(seed):
    """The GPU atomic-policy parity tests only mean something if the compiler really takes the
    atom path for them (incl. label-selector templates): every policy must lower."""
    g = Gen(5000 + seed)
    n = g.r.randint(1, 40)
    img = cedargpu.build_image([cedargpu.MemoryStore("a.cedar", g.atomic_policies(n))])
    st = cedargpu.image_stats(img)
    assert st["policies"] == n and st["atomic"] == n, st


def test_c3_workload_is_fully_atomic():
    from cedargpu import synth
    pop = synth.Population(seed=7)
    img = cedargpu.build_image([cedargpu.MemoryStore("c3.cedar", synth.abac_policies(2000, seed=31, pop=pop))])
    st = cedargpu.image_stats(img)
    assert st["atomic"] == st["policies"] == 2000, st


# ------------------------------------------------------------------ delta images (§8 f2)
def _tenant_docs(n_pol=4000, n_ns=40, seed=51):
    tpop = synth.Population(seed=7, n_namespaces=n_ns)
    return synth.multitenant_policies(n_pol, seed=seed, pop=tpop)


def test_delta_one_document_edit_is_small_and_exact():
    """A one-CRD edit (crd.go:62 update event) through the incremental compiler: the delta is a
    small fraction of the image and base + delta reproduces the new blob byte for byte."""
    docs = _tenant_docs()
    comp = cedargpu.Compiler()
    try:
        a = comp.build([cedargpu.CRDStore(docs)], epoch=1)
        docs[7] = (docs[7][0], docs[7][1], docs[7][2].replace("permit", "forbid", 1))
        b = comp.build([cedargpu.CRDStore(docs)], epoch=2)
        docs.append(("new-tenant", "new.cedar", 'permit(principal, action == k8s::Action::"get", resource);'))
        c = comp.build([cedargpu.CRDStore(docs)], epoch=3)
    finally:
        comp.close()
    # an edited document: < 1 % of the image; an added one (every later head index moves: word
    # fixups for the scope-index entries, the bitset values re-sent) < 10 %
    for base, new, frac in ((a, b, 0.01), (b, c, 0.10), (a, c, 0.10)):
        d = cedargpu.image_delta(base, new)
        info = cedargpu.delta_info(d)
        assert info["base_len"] == len(base) and info["new_len"] == len(new)
        assert len(d) < frac * len(new), (len(d), len(new))
        assert cedargpu.image_patch(base, d) == new
    # identical images: copies only (the header's epoch aside)
    d = cedargpu.image_delta(a, a)
    assert cedargpu.delta_info(d)["literal_bytes"] == 0 and cedargpu.image_patch(a, d) == a


def test_delta_arbitrary_bytes_and_rejections():
    import random
    rnd = random.Random(5)
    base = bytes(rnd.getrandbits(8) for _ in range(50_000))
    # an insertion, a deletion and an overwrite: the shifts are found again
    new = base[:1000] + b"inserted" * 40 + base[1000:20_000] + base[21_000:40_000] + b"\x00" * 300 + base[40_300:]
    d = cedargpu.image_delta(base, new)
    assert cedargpu.image_patch(base, d) == new
    assert cedargpu.delta_info(d)["literal_bytes"] < 2000
    for b2, n2 in ((b"", b"abc"), (b"abc", b""), (b"", b""), (base, base[::-1])):
        assert cedargpu.image_patch(b2, cedargpu.image_delta(b2, n2)) == n2
    # another base (length), a flipped literal byte (checksum), truncation, a bad magic
    with pytest.raises(cedargpu.CedarGPUError):
        cedargpu.image_patch(base[:-1], d)
    lit_at = len(d) - 1
    bad = bytearray(d)
    bad[lit_at] ^= 1
    with pytest.raises(cedargpu.CedarGPUError):
        cedargpu.image_patch(base, bytes(bad))
    with pytest.raises(cedargpu.CedarGPUError):
        cedargpu.image_patch(base, d[:-5])
    with pytest.raises(ValueError):
        cedargpu.delta_info(b"XXXX" + d[4:])
    # an operation pointing outside the base
    bad = bytearray(d)
    bad[56 + 16:56 + 24] = (len(base) + 10).to_bytes(8, "little")  # the first operation's src
    with pytest.raises(cedargpu.CedarGPUError):
        cedargpu.image_patch(base, bytes(bad))


def test_two_step_build_writes_the_same_blob():
    """cg_compiler_build_sized + cg_compiler_write_image (Compiler.build's path: the blob serialized
    straight into the caller's buffer, sections of >= 1 MB copied on several threads) gives the
    bytes cg_compiler_build returns; a write without a held image, or into a short buffer, fails."""
    import ctypes
    lib = cedargpu._lib.lib
    pop = synth.Population(seed=3, n_users=200, n_groups=40)
    text = synth.abac_policies(3000, seed=9, pop=pop)
    c = cedargpu.Compiler()
    two = c.build([cedargpu.MemoryStore("p.cedar", text)], epoch=5, entities=pop.static_entities())
    c.close()
    assert len(two) > (1 << 20)  # past the deferred-copy size
    c = cedargpu.Compiler()
    c.build([cedargpu.MemoryStore("p.cedar", text)], epoch=5, entities=pop.static_entities())  # same documents held
    out, n = ctypes.c_void_p(), ctypes.c_size_t(0)
    assert lib.cg_compiler_build(c._h, 5, ctypes.byref(out), ctypes.byref(n)) == 0
    one = ctypes.string_at(out, n.value)
    lib.cg_free(out)
    assert one == two
    buf = ctypes.create_string_buffer(16)
    assert lib.cg_compiler_write_image(c._h, buf, 16) != 0  # nothing held
    assert lib.cg_compiler_build_sized(c._h, 5, ctypes.byref(n)) == 0
    assert lib.cg_compiler_write_image(c._h, buf, 16) != 0  # too short
    big = ctypes.create_string_buffer(n.value)
    assert lib.cg_compiler_write_image(c._h, big, n.value) == 0
    assert big.raw == two
    c.close()


def test_duplicate_class_table_survives_the_blob():
    """The image's host-side duplicate-class table (image.h RS_CLASS: the host lists a class the
    candidate pass reports by its representative) is the blob's tail: an image with classes loads,
    a rebuild writes it again, and a member index past the policies is refused at load."""
    dup = "\n".join('forbid (principal, action == A::"w", resource) when { resource.owner != principal.name };'
                    for _ in range(150))
    singles = "\n".join(f'permit (principal, action == A::"r", resource) when {{ resource.level == {i} }};' for i in range(50))
    likes = 'permit (principal, action == A::"l", resource) when { resource.name like "prod-*" };\n' \
            'permit (principal, action == A::"l", resource) when { resource.path like "/a*b*c" };'
    stores = [cedargpu.MemoryStore("a.cedar", dup), cedargpu.MemoryStore("b.cedar", singles), cedargpu.MemoryStore("c.cedar", likes)]
    img = cedargpu.build_image(stores, epoch=3)
    assert cedargpu.index_stats(img)["entries"] > 0
    assert cedargpu.build_image(stores, epoch=3) == img
    n_pol = 202
    # the tail: [n, class offsets (n_pol + 1)] [n, members (n_pol)]; the last member, past the set
    assert int.from_bytes(img[-4 * (n_pol + 1):-4 * n_pol], "little") == n_pol
    bad = bytearray(img)
    bad[-4:] = (n_pol + 5).to_bytes(4, "little")
    with pytest.raises(ValueError):  # (deserialize: "corrupt image (duplicate classes)")
        cedargpu.index_stats(bytes(bad))

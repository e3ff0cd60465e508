"""Incremental compiler (cg_compiler_clear, the parse cache and the lowered-document cache, §8(f)
rank 2): a rebuild after a store change parses and lowers only the new or changed documents. With
incremental lowering off every build is byte-identical to a fresh compiler's; with it on (the
default) a rebuild copies the unchanged documents' lowered policies, falls back to a full build when
an image-wide choice changes, and its image holds the same policies in the same order (the GPU
suite checks that it decides every request as the fresh image does: tests/test_gpu_parity.py).
Host only."""
import json
import cedargpu
from cedargpu import synth


def _tenants(n_docs, per_doc, seed):
    pop = synth.Population(seed=seed, n_users=500, n_groups=60)
    text = synth.abac_policies(n_docs * per_doc, seed=seed, pop=pop)
    pols = [p for p in text.split("\n\n") if p.strip()]
    return [(f"tenant-{i:04d}", f"uid-{i}", "\n\n".join(pols[i * per_doc:(i + 1) * per_doc])) for i in range(n_docs)]


def _fresh(stores, epoch):
    return cedargpu.build_image(stores, epoch=epoch)


def test_rebuild_after_crd_changes_is_identical_to_a_fresh_build():
    docs = _tenants(60, 20, seed=5)
    comp = cedargpu.Compiler(incremental=False)
    img1 = comp.build([cedargpu.CRDStore(docs)], epoch=1)
    assert img1 == _fresh([cedargpu.CRDStore(docs)], 1)
    assert comp.cache_stats() == {"hits": 0, "misses": 60, "entries": 60}

    # one CRD updated, one removed, one added (crd.go:62,85,102,114 events)
    changed = list(docs)
    changed[7] = (changed[7][0], changed[7][1], changed[7][2].replace("permit", "forbid", 1))
    del changed[20]
    changed.append(("tenant-new", "uid-new", docs[3][2]))
    img2 = comp.build([cedargpu.CRDStore(changed)], epoch=2)
    assert img2 == _fresh([cedargpu.CRDStore(changed)], 2)
    st = comp.cache_stats()
    # tenant-new reuses tenant-0003's text under another name: a different document
    assert (st["hits"], st["misses"]) == (58, 2)
    assert st["entries"] == 60  # the removed and the superseded text are dropped
    assert img2 != img1
    comp.close()


def test_rebuild_with_tiers_and_static_policy():
    docs = _tenants(10, 10, seed=9)
    stores = [cedargpu.MemoryStore("base.cedar", synth.abac_policies(50, seed=2)), cedargpu.CRDStore(docs),
              cedargpu.ALLOW_ALL_ADMISSION]
    comp = cedargpu.Compiler(incremental=False)
    a = comp.build(stores, epoch=3)
    b = comp.build(stores, epoch=3)
    assert a == b == _fresh(stores, 3)
    assert comp.cache_stats()["misses"] == 0
    comp.close()


def test_syntax_error_reports_and_keeps_cache_usable():
    """A memory store's document that does not parse fails the build (memory.go:17-22); the
    compiler's cache stays usable."""
    docs = _tenants(5, 5, seed=4)
    text = "\n".join(d[2] for d in docs)
    comp = cedargpu.Compiler(incremental=False)
    comp.build([cedargpu.MemoryStore("m.cedar", text)], epoch=1)
    try:
        comp.build([cedargpu.MemoryStore("m.cedar", text + "\npermit (principal, action, resource) when { ;")], epoch=2)
        raise AssertionError("expected a compile error")
    except cedargpu.CompileError:
        pass
    assert comp.build([cedargpu.MemoryStore("m.cedar", text)], epoch=1) == _fresh([cedargpu.MemoryStore("m.cedar", text)], 1)
    comp.close()


def test_broken_crd_is_skipped_and_other_edits_apply():
    """crd.go:51-55 / 83-95: a CRD whose content does not parse is logged and contributes no
    policies -- an update that breaks it drops its old ones -- while every other CRD loads and
    later edits to them take effect. The same holds for directory files (directory.go:69-73) and
    AVP statements (verified_permissions.go:89-93)."""
    docs = _tenants(6, 5, seed=6)
    comp = cedargpu.Compiler(incremental=False)
    img1 = comp.build([cedargpu.CRDStore(docs)], epoch=1)
    assert comp.doc_errors() == []
    broken = list(docs)
    broken[2] = (broken[2][0], broken[2][1], "permit (principal, action, resource) when { ;")
    broken[4] = (broken[4][0], broken[4][1], broken[4][2].replace("permit", "forbid", 1))  # another CRD's edit
    img2 = comp.build([cedargpu.CRDStore(broken)], epoch=2)
    errs = comp.doc_errors()
    assert [e["filename"] for e in errs] == [docs[2][0]] and errs[0]["error"]
    without = [d for k, d in enumerate(broken) if k != 2]
    assert img2 == _fresh([cedargpu.CRDStore(without)], 2)
    assert cedargpu.image_stats(img2)["policies"] == cedargpu.image_stats(img1)["policies"] - 5
    # directory and AVP stores skip the same way; a memory store does not
    files = {"a.cedar": docs[0][2], "b.cedar": "forbid (principal,", "c.cedar": docs[1][2]}
    img3 = comp.build([cedargpu.DirectoryStore(files)], epoch=3)
    assert [e["filename"] for e in comp.doc_errors()] == ["b.cedar"]
    assert img3 == _fresh([cedargpu.DirectoryStore({k: v for k, v in files.items() if k != "b.cedar"})], 3)
    img4 = comp.build([cedargpu.AVPStore([("p1", docs[0][2]), ("p2", "permit (")])], epoch=4)
    assert img4 == _fresh([cedargpu.AVPStore([("p1", docs[0][2])])], 4)
    comp.close()


def _meta(img):
    """(id, tier, forbid) of every policy in image order, and the image's shape."""
    st = cedargpu.image_stats(img)
    return st["policies"], st["tiers"], st["atomic"], st["hot"]


def test_incremental_rebuild_lowers_only_changed_documents():
    docs = _tenants(60, 20, seed=5)
    comp = cedargpu.Compiler()
    img1 = comp.build([cedargpu.CRDStore(docs)], epoch=1)
    assert img1 == _fresh([cedargpu.CRDStore(docs)], 1)  # the first build is a full one
    lb = comp.last_build()
    assert lb["incremental"] is False and lb["why_full"] == "first build" and lb["lowered"] == 1200
    # one CRD updated, one removed, one added (crd.go:62,85,102,114 events)
    changed = list(docs)
    changed[7] = (changed[7][0], changed[7][1], changed[7][2].replace("permit", "forbid", 1))
    del changed[20]
    changed.append(("tenant-new", "uid-new", docs[3][2]))
    img2 = comp.build([cedargpu.CRDStore(changed)], epoch=2)
    lb = comp.last_build()
    assert lb["incremental"] is True and lb["lowered"] == 40 and lb["reused"] == 1160
    fresh2 = _fresh([cedargpu.CRDStore(changed)], 2)
    assert img2 != fresh2  # the removed document's words stay in the arenas
    assert _meta(img2) == _meta(fresh2)
    # the same documents again: nothing to lower
    assert comp.build([cedargpu.CRDStore(changed)], epoch=3) and comp.last_build()["lowered"] == 0
    comp.close()


def test_incremental_falls_back_to_full_builds():
    docs = _tenants(20, 10, seed=8)
    comp = cedargpu.Compiler()
    comp.build([cedargpu.CRDStore(docs)], epoch=1)
    # a new document whose conditions read a path used more than any other: the hot paths change
    heavy = "\n".join(f'permit (principal, action, resource) when {{ context.zzz{k % 3} == {k} && context.zzz{k % 3} != 5 }};'
                      for k in range(400))
    img = comp.build([cedargpu.CRDStore(docs + [("heavy", "uid-h", heavy)])], epoch=2)
    lb = comp.last_build()
    assert lb["incremental"] is False and lb["why_full"] == "hot attribute paths changed"
    assert img == _fresh([cedargpu.CRDStore(docs + [("heavy", "uid-h", heavy)])], 2)
    # new static entities: a full build
    ents = [{"uid": {"type": "k8s::Group", "id": "g1"}, "attrs": {}, "parents": []}]
    comp.build([cedargpu.CRDStore(docs)], epoch=3, entities=ents)
    assert comp.last_build()["why_full"] in ("static entities changed", "hot attribute paths changed")
    comp.build([cedargpu.CRDStore(docs)], epoch=4, entities=ents)
    assert comp.last_build()["incremental"] is True
    comp.close()


def test_incremental_compacts_after_churn():
    """Every document replaced again and again: the arenas' garbage triggers a full build, whose
    image is byte-identical to a fresh one."""
    docs = _tenants(10, 10, seed=3)
    comp = cedargpu.Compiler()
    comp.build([cedargpu.CRDStore(docs)], epoch=1)
    modes = []
    for r in range(6):
        docs = [(n, u, t + f"\n// edit {r}\n") for n, u, t in docs]
        img = comp.build([cedargpu.CRDStore(docs)], epoch=2 + r)
        lb = comp.last_build()
        modes.append(lb["incremental"])
        if not lb["incremental"]:
            assert lb["why_full"] == "compaction"
            assert img == _fresh([cedargpu.CRDStore(docs)], 2 + r)
    assert True in modes and False in modes
    comp.close()


def test_incremental_with_repeated_policy_ids():
    """PolicySet.Add replaces a repeated ID in place (an AVP store listing one ID twice): the
    replaced policy drops out of the image, in full and in incremental builds alike."""
    t = _tenants(4, 1, seed=11)
    stmts = [("p1", t[0][2]), ("p2", t[1][2]), ("p1", t[2][2])]
    comp = cedargpu.Compiler()
    comp.build([cedargpu.AVPStore(stmts), cedargpu.CRDStore(t[3:])], epoch=1)
    stores2 = [cedargpu.AVPStore(stmts + [("p3", t[3][2])]), cedargpu.CRDStore(t[3:])]
    img = comp.build(stores2, epoch=2)
    assert comp.last_build()["incremental"] is True
    assert _meta(img) == _meta(_fresh(stores2, 2)) and _meta(img)[0] == 4
    comp.close()


def test_incremental_keeps_contains_slots_out_of_prefix_keys():
    """A slot a contains atom reads carries element hashes, so the scope index never files `like
    "lit*"` prefix keys on it (image.h "prefix level-2 keys"). An incremental build that adds
    prefix-pattern policies on such a slot must make the same choice as a fresh build: its index
    shape (list-keyed slots, prefix-keyed slots, entries) equals the fresh image's."""
    base = "\n".join(f'permit (principal, action == k8s::Action::"get", resource) when {{ context.tags.contains("t{k}") }};'
                     for k in range(40))
    base += "\n" + "\n".join(f'permit (principal, action == k8s::Action::"list", resource) when {{ context.path like "/p{k}*" }};'
                             for k in range(40))
    extra = "\n".join(f'forbid (principal, action == k8s::Action::"get", resource) when {{ context.tags like "x{k}*" }};'
                      for k in range(5))
    docs = [("a", "uid-a", base)]
    comp = cedargpu.Compiler()
    comp.build([cedargpu.CRDStore(docs)], epoch=1)
    docs2 = docs + [("b", "uid-b", extra)]
    img = comp.build([cedargpu.CRDStore(docs2)], epoch=2)
    assert comp.last_build()["incremental"] is True
    fresh = _fresh([cedargpu.CRDStore(docs2)], 2)
    got, want = cedargpu.index_stats(img), cedargpu.index_stats(fresh)
    assert want["cslot_mask"] != 0 and want["pslot_mask"] != 0          # both kinds of list slots in use
    assert want["cslot_mask"] & want["pslot_mask"] == 0                 # never one slot for both
    assert got == want
    assert _meta(img) == _meta(fresh)
    comp.close()

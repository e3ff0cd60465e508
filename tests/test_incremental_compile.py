"""Incremental compiler (cg_compiler_clear + the parse cache, §8(f) rank 2): a rebuild after a store
change parses only the new or changed documents, and its image is byte-identical to a build by a
fresh compiler. Host only."""
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
    comp = cedargpu.Compiler()
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
    comp = cedargpu.Compiler()
    a = comp.build(stores, epoch=3)
    b = comp.build(stores, epoch=3)
    assert a == b == _fresh(stores, 3)
    assert comp.cache_stats()["misses"] == 0
    comp.close()


def test_syntax_error_reports_and_keeps_cache_usable():
    docs = _tenants(5, 5, seed=4)
    comp = cedargpu.Compiler()
    comp.build([cedargpu.CRDStore(docs)], epoch=1)
    bad = list(docs) + [("broken", "u", "permit (principal, action, resource) when { ;")]
    try:
        comp.build([cedargpu.CRDStore(bad)], epoch=2)
        raise AssertionError("expected a compile error")
    except cedargpu.CompileError:
        pass
    assert comp.build([cedargpu.CRDStore(docs)], epoch=1) == _fresh([cedargpu.CRDStore(docs)], 1)
    comp.close()

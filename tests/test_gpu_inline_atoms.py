"""GPU parity of the inline atoms (image.h AK_LIKEI, AK_INSTR): `like` patterns of at most one star
whose literals fit 8 bytes, and `[strings].contains(x)` of 1-3 strings, evaluated from the atom's own
words and the row's like words (staged with the hot values, or read from the string when not
staged: CEDARGPU_LIKE_STAGE=0), against the oracle on strings around the 8-byte edges, multi-byte
UTF-8, empty strings, non-string and missing attributes (type / attribute errors), on the one-launch
small-batch kernel and on the split first pass with its large stage."""
import json

import pytest

import cedar_oracle as co
import cedargpu

from test_gpu_parity import check_items, ctx, oracle_tiers  # noqa: F401  (module fixture)

pytestmark = pytest.mark.gpu

PATTERNS = ["", "a", "abcdefgh", "abcdefghi", "ab*", "abcdefgh*", "*gh", "*bcdefgh", "a*h", "abcd*efgh", "abc*fgh",
            "*", "**", "a**h", "é*", "*é", "x\\*y", "*\\**", "prod-*", "/healthz*", "ab*ba", "a*b*c"]
STRINGS = ["", "a", "ab", "aba", "abab", "abcdefg", "abcdefgh", "abcdefghi", "abcdefghijklmnop", "abcdefgh-abcdefgh",
           "aXh", "ah", "h", "é", "éé", "aéh", "x*y", "xy", "prod-", "prod-api", "/healthz", "/healthz/ready",
           "abba", "abcba", "abc"]


def _policies():
    out = []
    for p in PATTERNS:
        out.append(f'permit (principal, action == A::"like", resource) when {{ resource.name like "{p}" }};')
    out.append('forbid (principal, action == A::"like", resource) when { resource.n like "a*" };')  # type error on a long
    out.append('permit (principal, action == A::"like", resource) when { resource.missing like "a*" };')  # attribute error
    out.append('permit (principal, action == A::"like", resource) when { resource has opt && resource.opt like "*z" };')
    for s in (['"abc"'], ['"abc"', '"abcdefgh"'], ['"a"', '""', '"é"'], ['"a"', '"b"', '"c"', '"abc"']):
        out.append(f'permit (principal, action == A::"set", resource) when {{ [{", ".join(s)}].contains(resource.name) }};')
    out.append('permit (principal, action == A::"set", resource) when { ["1", "2"].contains(resource.n) };')  # non-string
    return "\n".join(out)


def _items():
    items = []
    for i, s in enumerate(STRINGS):
        for act in ("like", "set"):
            attrs = {"name": s, "n": 7}
            if i % 3 == 0:
                attrs["opt"] = s + "z"
            elif i % 3 == 1:
                attrs["opt"] = 5
            ents = [{"uid": {"type": "R", "id": f"r{i}"}, "attrs": attrs, "parents": []}]
            req = {"principal": {"type": "U", "id": "u"}, "action": {"type": "A", "id": act},
                   "resource": {"type": "R", "id": f"r{i}"}, "context": {}}
            items.append((ents, req))
    # a resource absent from the entity map: every attribute access errors
    items.append(([], {"principal": {"type": "U", "id": "u"}, "action": {"type": "A", "id": "like"},
                       "resource": {"type": "R", "id": "none"}, "context": {}}))
    return items


@pytest.mark.parametrize("words", ["0", "1"])
@pytest.mark.parametrize("stage", ["1", "0"])
@pytest.mark.parametrize("small_n", [None, "0"])
def test_inline_like_and_string_sets(ctx, stage, small_n, words, monkeypatch):  # noqa: F811
    """words=1 builds the image with row like words (CEDARGPU_LIKE_WORDS, read by the compiler per
    build): the encoder writes each like slot's length and first / last 8 bytes into the row, and
    with stage=1 the probe kernels stage them behind the hot values (the compact candidate pass's
    16-entry hot rows hold them here), so AK_LIKEI reads LDS; stage=0 reads the string's bytes."""
    monkeypatch.setenv("CEDARGPU_LIKE_STAGE", stage)
    monkeypatch.setenv("CEDARGPU_LIKE_WORDS", words)
    if small_n is not None:
        monkeypatch.setenv("CEDARGPU_SMALL_N", small_n)
    stores = [cedargpu.MemoryStore("inline.cedar", _policies())]
    st = cedargpu.image_stats(cedargpu.build_image(stores))
    assert (st["row_like_slots"] > 0) == (words == "1")
    items = _items() * 3  # (past the small path's tiny batches; the split pass's wave pooling)
    check_items(ctx, stores, items)


def test_like_words_mixed_incremental_build(ctx, monkeypatch):  # noqa: F811
    """an image compiled without row like words, then rebuilt incrementally with
    CEDARGPU_LIKE_WORDS=1 for one new document: that document's inline like atoms mark their slot
    in the image's like slots, while the kept documents' atoms on other slots were lowered without
    staged words. The device reads staged words only for a slot whose bit is set, so every request
    still decides as the oracle does, on both first-pass paths."""
    base = _policies()  # (its resource.opt atom keeps the hot slots of a fresh build: incremental)
    extra = 'permit (principal, action == A::"like", resource) when { resource has opt && resource.opt like "ab*" };'
    s1 = [cedargpu.MemoryStore("inline.cedar", base)]
    s2 = [cedargpu.MemoryStore("inline.cedar", base), cedargpu.MemoryStore("extra.cedar", extra)]
    monkeypatch.setenv("CEDARGPU_LIKE_WORDS", "0")
    comp = cedargpu.Compiler(incremental=True)
    try:
        comp.build(s1, epoch=901)
        monkeypatch.setenv("CEDARGPU_LIKE_WORDS", "1")
        img = comp.build(s2, epoch=902)
        assert comp.last_build()["incremental"]
    finally:
        comp.close()
    assert cedargpu.image_stats(img)["row_like_slots"] == 1  # resource.opt only (the new document's)
    ctx.load(img, 902)
    items = _items() * 3
    otiers = oracle_tiers(s2)
    for small_n in ("0", "2048"):
        monkeypatch.setenv("CEDARGPU_SMALL_N", small_n)
        b = ctx.batch()
        b.add_json(json.dumps([{"entities": e, "request": r} for e, r in items]))
        b.submit()
        b.wait()
        for i, (ents, req) in enumerate(items):
            want_ok, want_diag, _ = co.tiered_is_authorized(otiers, co.entities_from_json(ents), co.request_from_json(req))
            assert b.decision(i)[0] == want_ok and b.diagnostic(i) == want_diag.to_go_json(), (small_n, req)
        b.close()

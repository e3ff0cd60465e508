"""GPU parity of the inline atoms (image.h AK_LIKEI, AK_INSTR): `like` patterns of at most one star
whose literals fit 8 bytes, and `[strings].contains(x)` of 1-3 strings, evaluated from the atom's own
words and the row's like words (staged with the hot values, or read from the string when not
staged: CEDARGPU_LIKE_STAGE=0), against the oracle on strings around the 8-byte edges, multi-byte
UTF-8, empty strings, non-string and missing attributes (type / attribute errors), on the one-launch
small-batch kernel and on the split first pass with its large stage."""
import pytest

import cedargpu

from test_gpu_parity import check_items, ctx  # noqa: F401  (module fixture)

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


@pytest.mark.parametrize("stage", ["1", "0"])
@pytest.mark.parametrize("small_n", [None, "0"])
def test_inline_like_and_string_sets(ctx, stage, small_n, monkeypatch):  # noqa: F811
    monkeypatch.setenv("CEDARGPU_LIKE_STAGE", stage)
    if small_n is not None:
        monkeypatch.setenv("CEDARGPU_SMALL_N", small_n)
    items = _items() * 3  # (past the small path's tiny batches; the split pass's wave pooling)
    check_items(ctx, [cedargpu.MemoryStore("inline.cedar", _policies())], items)

"""The shapes of tests/lowering_cases.py compile to device images (no CG_E_COMPILE for valid Cedar
within the documented limits) and the two oracles agree on them; GPU parity is in
tests/test_gpu_parity.py (test_lowered_shapes_vs_oracle)."""
import os

import pytest

import cedar_oracle as co
import cedargpu
from lowering_cases import CASES
from test_oracle_cxx import _compare


@pytest.mark.parametrize("name", sorted(CASES))
def test_lowered_shapes_compile(name):
    docs, _ = CASES[name]()
    for fname, text in docs:
        img = cedargpu.build_image([cedargpu.MemoryStore(fname, text)])
        st = cedargpu.image_stats(img)
        assert st["policies"] == len(co.parse_policies(text, fname)), st


@pytest.mark.parametrize("name", sorted(CASES))
def test_lowered_shapes_oracles_agree(name):
    docs, items = CASES[name](n=120)
    _compare([docs], items)


def test_unknown_functions_and_methods_are_parse_errors():
    """Both parsers reject names Cedar does not define, so the whole document is rejected (or
    skipped by the stores that skip bad documents) instead of failing one policy at run time."""
    for src in ['permit (principal, action, resource) when { foo("x") };',
                'permit (principal, action, resource) when { ip("1.2.3.4", "x") == ip("1.2.3.4") };',
                'permit (principal, action, resource) when { context.s.frobnicate() };',
                'permit (principal, action, resource) when { context.s.contains() };',
                'permit (principal, action, resource) when { ip("::1").isIpv4(1) };']:
        with pytest.raises(co.ParseError):
            co.parse_policies(src, "x.cedar")
        with pytest.raises(cedargpu.CompileError):
            cedargpu.build_image([cedargpu.MemoryStore("x.cedar", src)])


def test_nesting_beyond_64_slots_is_a_named_limit():
    deep = "context.a"
    for _ in range(70):
        deep = f"1 + ({deep})"
    with pytest.raises(cedargpu.CompileError, match="64 registers"):
        cedargpu.build_image([cedargpu.MemoryStore("x.cedar", f"permit (principal, action, resource) when {{ {deep} > 0 }};")])


def test_contains_shapes_index_and_oracles_agree():
    import contains_cases as cc
    img = cedargpu.build_image([cedargpu.MemoryStore("c.cedar", cc.POLICIES)])
    st = cedargpu.image_stats(img)
    assert st["indexed"] and st["policies"] == st["atomic"] == 12, st
    _compare([[("c.cedar", cc.POLICIES)]], cc.items(300))


def test_inline_like_and_string_set_atoms_index():
    """The inline atoms (image.h AK_LIKEI / AK_INSTR) keep a policy atomic and indexed, and an inline
    `like` with a literal prefix still files a prefix key (tests/test_gpu_inline_atoms.py runs them)."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from test_gpu_inline_atoms import _policies
    img = cedargpu.build_image([cedargpu.MemoryStore("inline.cedar", _policies())], epoch=1)
    st = cedargpu.image_stats(img)
    assert st["atomic"] == st["policies"] and st["indexed"], st
    ix = cedargpu.index_stats(img)
    assert ix["pslot_mask"], ix  # `like "ab*"` etc.: prefix keys on resource.name

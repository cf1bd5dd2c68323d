"""The executable spec model (tests/golden/spec_model.py) on its own: the
pieces it takes from the reference's definitions, and (where the reference
is present) a full regeneration of the committed spec fixtures."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import spec_model as S  # noqa: E402

REF = os.environ.get("VIGOR_REF", "/root/reference")


def test_generated_hash_kat():
    """FlowId_hash(1, 2, 3, 4, 5, 6) = 0xae93f0ff (SURVEY.md KAT)."""
    assert S.struct_hash(1, 2, 3, 4, 5, 6) == 0xAE93F0FF


def test_emap_expiry_is_strictly_below_cutoff():
    em = S.Emap(4)
    em.add("a", S.Emap.AUTO, 10)
    em.add("b", S.Emap.AUTO, 20)
    em.expire_all(20)  # is_cell_expired: ts < time
    assert not em.has("a") and em.has("b")


def test_emap_dchain_order_and_lru():
    """Fresh indices in order, freed ones last-freed first; expiry frees in
    LRU order (a refresh moves an index to the young end)."""
    em = S.Emap(4)
    for k, t in zip("abcd", (1, 2, 3, 4)):
        em.add(k, S.Emap.AUTO, t)
    assert [em.get(k) for k in "abcd"] == [0, 1, 2, 3] and em.full()
    em.refresh_idx(em.get("a"), 5)
    em.expire_all(5)  # frees b, c, d (LRU first); a was refreshed
    assert em.has("a") and not em.has("b")
    em.add("e", S.Emap.AUTO, 6)
    assert em.get("e") == 3  # the last one freed
    em.erase("a")
    em.add("f", S.Emap.AUTO, 7)
    assert em.get("f") == 0


def test_cht_choice_takes_first_live_backend_of_the_row():
    em = S.Emap(3)
    cht = [2, 0, 1, 1, 2, 0]  # height 2, three backends per row
    em.add("x", S.Emap.AUTO, 1)  # backend index 0
    assert em.exists_with_cht(cht, 4) and em.choose_with_cht(cht, 4) == 0
    em.add("y", S.Emap.AUTO, 1)  # backend 1
    assert em.choose_with_cht(cht, 5) == 1


def test_spec_integer_division():
    code = S.compile_spec("return ([7 / 2], [])\n")
    assert S.run_packet(code, {}, {}) == ([3], [])


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "vignat")),
                    reason="reference absent (the fixtures carry its answers)")
def test_spec_fixtures_regenerate(tmp_path, monkeypatch):
    """make_spec_golden.py over the reference's spec.py files reproduces the
    committed fixtures (its own asserts check the oracle on every packet)."""
    import make_spec_golden as M
    monkeypatch.setattr(M, "HERE", str(tmp_path))
    M.main()
    for nf in ("nat", "fw", "bridge", "pol", "lb"):
        new = np.load(tmp_path / ("spec_%s.npz" % nf))
        old = np.load(os.path.join(HERE, "golden", "spec_%s.npz" % nf))
        for k in old.files:
            assert np.array_equal(new[k], old[k]), (nf, k)


@pytest.mark.parametrize("text", [
    "import os\nreturn ([], [])\n",
    "from os import system\n",
    "x = ether.__class__\n",
    "__import__('os')\n",
    "f = lambda: 1\n",
    "for i in [1]:\n    pass\n",
    "return ([open], [])\n" + "x = 'text'\n",
    "return [y for y in [1]]\n",
    "(pop_header)(ether, on_mismatch=([], []))\n" + "x = [1][0]()\n",
])
def test_spec_sandbox_rejects(text):
    """The spec files are untrusted text: anything outside the specs'
    vocabulary is refused before it is compiled, let alone run."""
    with pytest.raises(S.SpecRejected):
        S.compile_spec(text)


def test_spec_runs_without_builtins():
    code = S.compile_spec("return ([open], [])\n")
    with pytest.raises(NameError):
        S.run_packet(code, {}, {})

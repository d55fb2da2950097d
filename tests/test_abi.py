"""The C-ABI library loads without a GPU and exports every symbol include/splink_hip.h declares."""
import os
import re

from conftest import ROOT

from splink_amd import _native as N


def declared_functions():
    text = open(os.path.join(ROOT, "include", "splink_hip.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(spk_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for required in ("spk_ctx_create", "spk_block", "spk_gammas", "spk_em_histogram", "spk_em_finalize",
                     "spk_score", "spk_tf_apply", "spk_jaro_winkler_sim"):
        assert required in names


def test_library_exports_every_declared_symbol():
    lib = N.load_library()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(N.EXPORTS) == set(declared_functions())


def test_struct_layouts_match_header():
    assert N.OPERAND_DTYPE.itemsize == 40
    assert N.INSTR_DTYPE.itemsize == 32
    assert N.PROGRAM_DTYPE.itemsize == 16


def test_no_device_means_loud_failure():
    if N.device_count() > 0:
        return
    import pytest
    with pytest.raises(N.NativeUnavailable):
        N.Context(0)

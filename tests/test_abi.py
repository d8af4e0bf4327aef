"""The C-ABI library loads and exports every symbol include/nst_hip.h declares (no GPU needed)."""
import ctypes
import os
import re

from conftest import REPO
from neuralstyletransferv1_amd import _lib


def _declared():
    src = open(os.path.join(REPO, "include", "nst_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nst_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert sorted(_lib.EXPORTED_SYMBOLS) == _declared()


def test_library_exports_every_declared_symbol():
    lib = _lib.lib()
    for name in _declared():
        assert hasattr(lib, name), name
    assert lib.nst_version().decode().startswith("nst_hip")


def test_argument_validation_without_gpu():
    lib = _lib.lib()
    h = ctypes.c_void_p()
    assert lib.nst_create(7, None, 0, 0, 0, ctypes.byref(h)) == -1
    assert b"invalid" in lib.nst_last_error()
    oh, ow = ctypes.c_int(), ctypes.c_int()
    assert lib.nst_output_hw(None, 8, 8, ctypes.byref(oh), ctypes.byref(ow)) == -1
    assert lib.nst_forward(None, None, 0, 1, 8, 8, 0, None, 0, None, 0, None) == -1
    assert lib.nst_gram(None, 0, 0, 1, 1, 1, None, None, 0, None) == -1


def test_presets_table_matches_header():
    src = open(os.path.join(REPO, "include", "nst_hip.h")).read()
    for name, val in _lib.PRESETS.items():
        assert re.search(rf"#define NST_PRESET_{name.upper()} {val}\b", src), name


def test_arch_ids_match_header():
    src = open(os.path.join(REPO, "include", "nst_hip.h")).read()
    for name in ("JOHNSON", "NST", "RECONET", "RECONET_FRN"):
        val = getattr(_lib, f"NST_ARCH_{name}")
        assert re.search(rf"#define NST_ARCH_{name} {val}\b", src), name


def test_frn_checkpoint_names_match_reference_layout():
    # ReCoNet(frn=True) (model.py:18-60 with frn.py): FRN at the norm's index with weight / bias / eps,
    # TLU tau after activated layers and on every ResLayer; the engine looks these names up
    from neuralstyletransferv1_amd.model import ReCoNet
    sd = ReCoNet(frn=True).state_dict()
    assert sd["encoder.layers.0.layers.1.eps"].shape == (1,)
    assert sd["encoder.layers.0.layers.2.tau"].shape == (1, 48, 1, 1)
    assert sd["encoder.layers.3.activation.tau"].shape == (1, 192, 1, 1)
    assert "encoder.layers.3.branch.1.layers.2.tau" not in sd  # the branch's second layer has no TLU
    assert sd["decoder.layers.3.layers.2.tau"].shape == (1, 48, 1, 1)
    assert len(sd) == 80

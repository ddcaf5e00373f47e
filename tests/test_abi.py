"""CPU checks of the drop-in boundary: the C-ABI library loads and exports
every symbol include/kb2e_engine.h declares (no compute calls, no GPU)."""
import ctypes
import os

import pytest
import re
import subprocess

from conftest import ROOT
from kb2e_amd import engine


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "kb2e_engine.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(kb2e_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_the_binding_list():
    assert declared_symbols() == sorted(engine.EXPORTS)


def test_library_exports_every_declared_symbol():
    so = engine.LIB_PATH
    assert os.path.exists(so), "build the engine first (make)"
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (kb2e_[a-z_0-9]+)", out))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    lib = ctypes.CDLL(so)
    for s in declared_symbols():
        assert hasattr(lib, s)


def test_default_config_is_reference_defaults():
    cfg = engine.Config()
    engine.lib().kb2e_default_config(ctypes.byref(cfg))
    # common/constants.h:28-40
    assert (cfg.dim, cfg.learning_rate, cfg.margin, cfg.method, cfg.num_batches, cfg.distance) == \
        (100, 0.001, 1.0, 1, 100, 0)
    assert cfg.precision == 64 and cfg.sampler == engine.SAMPLER_GLIBC


def test_create_without_gpu_fails_loudly():
    if os.path.exists("/dev/kfd"):  # a GPU box: nothing to check
        pytest.skip("GPU present")
    try:
        engine.Engine("E", 20, 10, 2, batches=1)
    except engine.EngineError:
        return
    raise AssertionError("creating an engine without a GPU must raise")

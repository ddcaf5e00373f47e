"""CPU checks of the text formats: the "%.6lf" formatter and
the "%lf" fast-path parser that the device kernels run (kb2e_amd/csrc/textio.hpp,
shared host/device inline code) against glibc's snprintf / strtod -- the
functions behind the reference's fprintf / fscanf (common/trainer.cpp:109-127,
transr/trainer.cpp:88-113).  Exact byte / bit equality."""
import os
import subprocess

from conftest import ROOT


def test_formatter_and_parser_match_glibc():
    exe = os.path.join(ROOT, "bin", "textio_check")
    assert os.path.exists(exe), "build first (make)"
    for seed in (1, 7):
        out = subprocess.run([exe, "400000", str(seed)], capture_output=True, text=True, timeout=120)
        assert out.returncode == 0, out.stdout + out.stderr
        assert out.stdout.startswith("ok ")

"""The exact fast sqrt / reciprocal / division forms of romis_amd/csrc/device_math.h against the IEEE operations
on the GPU: every float for sqrt and reciprocal, 2^32 hashed pairs + edge cases (NaN, inf, guard ends) for the
double-reciprocal division (tests/hip/fastmath_check.hip)."""
import json
import os
import subprocess

import pytest

from romis_amd import build

TOOL = os.path.join(build.OUT, "tools", "fastmath_check")


def test_fastmath_tool_built():
    assert os.path.exists(TOOL), "python -m romis_amd.build builds the checker"


@pytest.mark.gpu
def test_fast_forms_bit_exact():
    r = subprocess.run([TOOL], capture_output=True, text=True, timeout=300)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0, out
    assert out["sqrt"]["checked"] == 1879048192 + 1 and out["sqrt"]["bad"] == 0          # every q in [2^-96, FLT_MAX], and +0
    assert out["rcp"]["checked"] == 4194304002 and out["rcp"]["bad"] == 0            # every |b| in [2^-125, 2^125]
    assert out["div"]["checked"] > 4_000_000_000 and out["div"]["bad"] == 0

"""Every launch-shape knob restir_set_tuning accepts (romis_amd/csrc/restir.cpp) has its library default in the A/B
tooling (scripts/kbench.py DEFAULTS: cfg_kbench.py resets the knobs a variant does not set to these), and the
defaults there equal the Tuning struct's (romis_amd/csrc/restir_types.h).  CPU only, source text."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# knobs that select timing / frame-slot behaviour, not a kernel's launch shape (the bench sets them itself)
NOT_SHAPES = {"mis.chunk", "timing.every", "timing.fence", "timing.mask"}


def _knobs():
    src = open(os.path.join(ROOT, "romis_amd", "csrc", "restir.cpp")).read()
    return dict(re.findall(r'std::strcmp\(key, "([a-z0-9_.]+)"\)\) t\.([a-z0-9_]+) = ', src))


def _tuning_defaults():
    src = open(os.path.join(ROOT, "romis_amd", "csrc", "restir_types.h")).read()
    body = src[src.index("struct Tuning {"):]
    body = body[:body.index("};")]
    return {m: int(v, 0) for m, v in re.findall(r"uint32_t ([a-z0-9_]+) = (0x[0-9A-Fa-f]+u?|\d+)u?;", body.replace("u;", ";"))}


def test_kbench_defaults_cover_every_knob():
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from kbench import DEFAULTS
    knobs = _knobs()
    assert knobs, "no knobs parsed"
    missing = sorted(k for k in knobs if k not in DEFAULTS and k not in NOT_SHAPES)
    assert not missing, f"scripts/kbench.py DEFAULTS lacks {missing}"
    fields = _tuning_defaults()
    for key, field in knobs.items():
        if key in DEFAULTS and field in fields:
            assert DEFAULTS[key] == fields[field], f"{key}: kbench {DEFAULTS[key]} vs Tuning::{field} {fields[field]}"

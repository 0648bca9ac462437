"""Regenerate the fixtures that pin the oracle's inputs against the reference's OWN code.

Builds oracle/_ref/dump_ref (oracle/Makefile `ref`: the reference's scene.cpp, mesh.cpp, image.cpp,
tiny_obj_loader.cc, texture.cpp and tone_mapping.cpp compiled unmodified from /root/reference, linked with
oracle/ref_harness/dump_ref.cpp), runs it on /root/reference/data and splits its output into
  romis_amd/scenes/prebuilt_scenes.json  -- loadScenePrebuilt() results (scene assets the product loads)
  tests/golden/ref_fixtures.json         -- regularLightGrid, exposureToneMapping, acquireTexel and glm primitive vectors
Floats are stored as IEEE-754 bit patterns.  Run in the build container only (needs /root/reference).
"""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = os.environ.get("ROMIS_REFERENCE", "/root/reference")


def main() -> int:
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref", f"REF={REF}"])
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "ref.json")
        subprocess.check_call([os.path.join(ROOT, "oracle", "_ref", "dump_ref"), os.path.join(REF, "data"), out])
        with open(out) as fh:
            d = json.load(fh)
    scenes = {"source": "loadScenePrebuilt (src/scene/scene.cpp:68-132) via oracle/_ref/dump_ref",
              "float_encoding": "ieee754-bits", "scenes": d["scenes"]}
    with open(os.path.join(ROOT, "romis_amd", "scenes", "prebuilt_scenes.json"), "w") as fh:
        json.dump(scenes, fh, separators=(",", ":"))
    fx = {"source": "oracle/_ref/dump_ref (reference scene.cpp / tone_mapping.cpp / vendored glm 0.9.9.9)",
          "float_encoding": "ieee754-bits",
          "light_grid": d["light_grid"], "tonemap": d["tonemap"], "glm": d["glm"], "texel": d["texel"]}
    with open(os.path.join(ROOT, "tests", "golden", "ref_fixtures.json"), "w") as fh:
        json.dump(fx, fh, separators=(",", ":"))
    return 0


if __name__ == "__main__":
    sys.exit(main())

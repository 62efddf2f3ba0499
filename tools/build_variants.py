"""Build A/B variants of libcpt.so in parallel:  python tools/build_variants.py name:DEF=1,DEF2=3 ...
Outputs build/ab/<name>.so (shipped to the GPU box with the tree; build/ is git-ignored)."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cpppathtracer_amd import build  # noqa: E402


def one(spec):
    name, _, defs = spec.partition(":")
    defines = [d for d in defs.split(",") if d]
    out = os.path.join(build.REPO_DIR, "build", "ab", f"{name}.so")
    build.build(out=out, defines=defines)
    return out


if __name__ == "__main__":
    with ThreadPoolExecutor(max_workers=4) as ex:
        for out in ex.map(one, sys.argv[1:]):
            print("built", out)

"""Builds libcpt.so (the HIP kernels + C-ABI + C++ API) in-tree for gfx950 with hipcc.

hipcc cross-compiles without a GPU, so this runs in the build container; the resulting .so
travels to the GPU box with the repo snapshot.
"""
import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_PATH = os.path.join(PKG_DIR, "libcpt.so")

SOURCES = [
    os.path.join(CSRC, "cpt_kernels.hip"),
    os.path.join(CSRC, "cpt_wavefront.hip"),
    os.path.join(CSRC, "cpt_capi.cpp"),
    os.path.join(CSRC, "cpt_scene.cpp"),
    os.path.join(CSRC, "cpt_host_bvh.cpp"),
    os.path.join(CSRC, "cpt_host_rng.cpp"),
    os.path.join(CSRC, "cpt_api.cpp"),
]
HEADERS = [
    os.path.join(CSRC, "cpt_device.hpp"),
    os.path.join(CSRC, "cpt_internal.hpp"),
    os.path.join(CSRC, "cpt_context.hpp"),
    os.path.join(CSRC, "cpt_host.hpp"),
    os.path.join(CSRC, "cpt_path.hpp"),
    os.path.join(CSRC, "cpt_stamps.hpp"),
    os.path.join(CSRC, "cpt_tuning.hpp"),
    os.path.join(CSRC, "cpt_dn_exp.hpp"),
    os.path.join(REPO_DIR, "include", "cpt.h"),
]

# Float semantics: no FMA contraction, IEEE f32 div/sqrt, no fast math,
# f32 denormals kept — each expression rounds exactly as written, as in the CPU oracle.
HIPCC_FLAGS = [
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-shared",
    "-ffp-contract=off",
    "-fno-fast-math",
    "-fhip-fp32-correctly-rounded-divide-sqrt",
    "-fno-gpu-flush-denormals-to-zero",
    "-Wall",
    "-Wno-unused-function",
    # no SLP vectorizer: it packs independent f32 ops into v_pk_* pairs, which needs operands as
    # register pairs; at the 4-wave (128-VGPR) budget that spilled 9 registers to scratch
    # (C4: 1490 vs 1392 Mpaths/s without it; each lane's arithmetic is unchanged)
    "-fno-slp-vectorize",
    # the machine scheduler tries several schedules per region and keeps the best one that holds
    # the occupancy target (round 5, profiles/r05/ab_sched_strategy_*.log: C4 +0.3 to +3.6% in six
    # interleaved pairs on two boxes, 1990 vs 1965 Mpaths/s on average; C2 / C3 / the display kernel unchanged;
    # iterative-ilp: C4 +2%, C2 / C3 -2%; max-ilp / max-memory-clause / iterative-minreg: no gain).
    # It spills a few VGPRs where the default did not (timed megakernel 8 B, k_denoise_rows 20 B),
    # with no measurable cost (profiles/r05/ab_display_sched.log).
    "-mllvm", "-amdgpu-sched-strategy=iterative-maxocc",
] + os.environ.get("CPT_EXTRA_HIPCC_FLAGS", "").split()


def _hipcc():
    for p in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if p and (os.path.isabs(p) and os.path.exists(p) or not os.path.isabs(p)):
            return p
    return "hipcc"


def _extra_sources():
    return [s for s in SOURCES if os.path.exists(s)]


def needs_build() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    deps = _extra_sources() + [h for h in HEADERS if os.path.exists(h)] + [os.path.abspath(__file__)]   # (the flags)
    deps += [os.path.join(REPO_DIR, "include", "cpppathtracer", f)
             for f in os.listdir(os.path.join(REPO_DIR, "include", "cpppathtracer"))] if os.path.isdir(
        os.path.join(REPO_DIR, "include", "cpppathtracer")) else []
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, out: str = None, defines=()) -> str:
    """Build libcpt.so; `out`/`defines` produce A/B variants: defines is a list of "NAME=VALUE"
    strings or a {NAME: VALUE} dict."""
    if isinstance(defines, dict):
        defines = [f"{k}={v}" for k, v in defines.items()]
    target = out or LIB_PATH
    if not force and out is None and not defines and not needs_build():
        return LIB_PATH
    os.makedirs(os.path.dirname(os.path.abspath(target)), exist_ok=True)
    tmp = target + ".tmp"
    cmd = [_hipcc(), *HIPCC_FLAGS, *[f"-D{d}" for d in defines], "-I", os.path.join(REPO_DIR, "include"), "-o", tmp,
           *_extra_sources()]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, target)
    return target


EXAMPLE_SRC = os.path.join(REPO_DIR, "examples", "headless_render.cpp")
EXAMPLE_BIN = os.path.join(REPO_DIR, "build", "bin", "cpt_headless")


def build_examples(force: bool = False, verbose: bool = False) -> str:
    """The reference-app-shaped headless driver, host C++ only (g++), linked to libcpt.so."""
    lib = build()
    if (not force and os.path.exists(EXAMPLE_BIN)
            and os.path.getmtime(EXAMPLE_BIN) > max(os.path.getmtime(EXAMPLE_SRC), os.path.getmtime(lib))):
        return EXAMPLE_BIN
    os.makedirs(os.path.dirname(EXAMPLE_BIN), exist_ok=True)
    cmd = ["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-pthread", "-I", os.path.join(REPO_DIR, "include"),
           "-o", EXAMPLE_BIN, EXAMPLE_SRC, lib, "-Wl,-rpath,$ORIGIN/../../cpppathtracer_amd"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return EXAMPLE_BIN


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_examples(force="--force" in sys.argv, verbose=True))

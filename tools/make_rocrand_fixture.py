"""Extract rocRAND's precomputed XORWOW jump tables (ROCm, not the reference) into
tests/golden/rocrand_xorwow_tables.npz so the RNG pin also runs where ROCm headers are absent."""
import os
import re

import numpy as np

HDR = "/opt/rocm/include/rocrand/rocrand_xorwow_precomputed.h"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                   "rocrand_xorwow_tables.npz")


def parse(text, name):
    m = re.search(r"static const unsigned int " + name + r"\[XORWOW_JUMP_MATRICES\]\[XORWOW_SIZE\] = \{(.*?)\};",
                  text, re.S)
    nums = re.findall(r"(\d+)U?", m.group(1))
    return np.array([int(x) for x in nums], dtype=np.uint64).astype(np.uint32).reshape(32, 800)


if __name__ == "__main__":
    t = open(HDR).read()
    np.savez_compressed(OUT, jump=parse(t, "h_xorwow_jump_matrices"), seq=parse(t, "h_xorwow_sequence_jump_matrices"))
    print("wrote", OUT)

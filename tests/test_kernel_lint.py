"""Source lint of the HIP kernels for compiler pitfalls found on this toolchain (CPU-only).

amdclang 22 (ROCm 7.2) lowers ``__builtin_bit_cast(T, v[i])`` on an ext-vector ELEMENT lvalue to a
read of element 0, whatever ``i`` is: the LL hand-off of the fp32 MLP epoch kernel silently summed
the wrong partial logits until the element reads went through ``__uint_as_float(v[i])`` (see
csrc/kernels/persist_common.h). Whole-vector or array-element casts (``bit_cast(uint2, arr[k])``
where ``arr`` is an array of vectors) are fine; a cast of ``x[a][b]`` or ``x.y`` is not.
"""

import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BAD = [
    re.compile(r"__builtin_bit_cast\([^,()]+,\s*[A-Za-z_][A-Za-z0-9_]*(\[[^\]]+\]){2,}\s*\)"),  # x[a][b]
    re.compile(r"__builtin_bit_cast\([^,()]+,\s*[A-Za-z_][A-Za-z0-9_]*\s*\.\s*[xyzw]\s*\)"),  # x.y
]


def test_no_bit_cast_of_vector_elements():
    hits = []
    for path in glob.glob(os.path.join(ROOT, "csrc", "**", "*.*"), recursive=True):
        if not path.endswith((".hip", ".h", ".cpp")):
            continue
        with open(path) as f:
            for n, line in enumerate(f, 1):
                if any(b.search(line) for b in BAD):
                    hits.append(f"{os.path.relpath(path, ROOT)}:{n}: {line.strip()}")
    assert not hits, "bit_cast of a vector element (miscompiled: reads element 0):\n" + "\n".join(hits)

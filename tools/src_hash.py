"""Hash of the HIP/C++ sources of libdm: ties a PMC summary to the code it
measured (bench.py only reports `traffic` from a summary of the same code)."""
import hashlib
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "distributed-autonomous-exploration-and-mapping_amd", "csrc")


def src_hash() -> str:
    h = hashlib.sha256()
    for f in sorted(os.listdir(CSRC)):
        if f.endswith((".hip", ".cpp", ".h")):
            h.update(f.encode())
            h.update(open(os.path.join(CSRC, f), "rb").read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(src_hash())

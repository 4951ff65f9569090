"""Per-kernel register / scratch summary of a hipcc -Rpass-analysis=kernel-resource-usage log:
    python scripts/res_usage.py <log> [substring ...]"""
import re
import subprocess
import sys

FILT = "c++filt"


def summary(path):
    out = {}
    for blk in open(path).read().split("Function Name: ")[1:]:
        name = blk.split(" ")[0]
        try:
            dem = subprocess.run([FILT, name], capture_output=True, text=True).stdout.strip() or name
        except OSError:
            dem = name
        g = lambda k: (re.search(k + r": (\S+)", blk) or [None, None])[1]  # noqa: E731
        out[dem] = dict(vgpr=g("VGPRs"), agpr=g("AGPRs"), scratch=g(r"ScratchSize \[bytes/lane\]"),
                        vspill=g("VGPRs Spill"), occ=g(r"Occupancy \[waves/SIMD\]"))
    return out


if __name__ == "__main__":
    keys = sys.argv[2:]
    for k, v in summary(sys.argv[1]).items():
        if not keys or any(s in k for s in keys):
            print(f"vgpr {v['vgpr']:>4} agpr {v['agpr']:>3} scratch {v['scratch']:>5} spill {v['vspill']:>4} occ {v['occ']}  {k[:150]}")

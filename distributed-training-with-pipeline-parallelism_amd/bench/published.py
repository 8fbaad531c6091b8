"""The reference's published throughput table (notebook cell 25,
nb:679-732): 9 (layers, heads) configs x P in {2, 4} x 3 schedules, tokens/s on a 10-core
CPU over gloo, fp32, batch 32 x seq 128, m = 4, 5 timed fwd+bwd steps."""
from typing import Dict, Optional, Tuple

SCHEDULES = ("GPipe", "1F1B", "Interleaved1F1B")
# L H P  GPipe  1F1B  Interleaved1F1B   (nb:679-732, in notebook order)
_ROWS = """4 4 2 3154.76 3238.24 3278.79
4 4 4 3606.48 3722.89 3545.62
4 8 2 3051.49 2995.72 3219.27
4 8 4 3333.58 3541.49 3409.60
4 12 2 2899.89 2966.34 3023.31
4 12 4 3249.43 3323.24 3235.95
8 4 2 1769.51 1773.75 1895.92
8 4 4 1928.99 2019.28 2169.55
8 8 2 1671.32 1649.53 1796.30
8 8 4 1675.15 1680.10 1739.43
8 12 2 1371.54 1511.65 1252.73
8 12 4 1608.81 1714.38 1751.59
12 4 2 1095.58 1168.28 1228.10
12 4 4 1259.14 1276.17 1265.39
12 8 2 1036.03 1097.85 1157.26
12 8 4 1165.24 1234.93 1173.06
12 12 2 915.56 986.30 1072.16
12 12 4 1063.27 1210.86 1147.74"""

PUBLISHED: Dict[Tuple[int, int, int, str], float] = {}
SOURCE_LINE: Dict[Tuple[int, int, int, str], int] = {}
for _i, _line in enumerate(_ROWS.splitlines()):
    _L, _H, _P, *_v = _line.split()
    for _j, (_s, _x) in enumerate(zip(SCHEDULES, _v)):
        PUBLISHED[(int(_L), int(_H), int(_P), _s)] = float(_x)
        SOURCE_LINE[(int(_L), int(_H), int(_P), _s)] = 679 + 3 * _i + _j

# the 9 (L, H) configs of the sweep (nb:346-349); L8 H8 (the ModelArgs default) first
CONFIGS = ((8, 8), (4, 4), (4, 8), (4, 12), (8, 4), (8, 12), (12, 4), (12, 8), (12, 12))


def published(L: int, H: int, P: int, schedule: str) -> Optional[float]:
    """Published tok/s of (L, H, P, schedule), or None (P not in {2, 4}: never run)."""
    return PUBLISHED.get((int(L), int(H), int(P), schedule))

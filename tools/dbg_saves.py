import sys
sys.path.insert(0, ".")
from tests.gpu_harness import Pair
p = Pair(G=40, R=3, save_cap=1024, max_props=4)
for r in range(3):
    o, e = p.round(k=1, tick=(r % 2 == 0), read_index=(r % 3 == 0), encode_saves=True)
    errs = p.check_saves()
    print("round", r, "fb", e.fallbacks, "errs", len(errs))
    ce = p.check()
    print("check", len(ce), ce[:4])
    for g, s, _, eb, ob in errs[:1]:
        print(g, s, "dev", eb[0].hex() if eb else None, eb[1] if eb else None)
        print(g, s, "orc", ob[0].hex() if ob else None, ob[1] if ob else None)

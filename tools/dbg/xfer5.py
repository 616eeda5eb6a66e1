"""debug: leader transfer requested at a follower, R = 5 (test_gpu_transfer
[5-0-follower]); prints the per-destination outbox differences of the first
round whose message counts differ."""
import sys
sys.path.insert(0, ".")
from dragonboat_amd import abi
from tests.gpu_harness import Pair, by_dest

R, G = 5, 24
p = Pair(G=G, R=R, elections=1, pre_vote=0)
for i in range(3):
    o, e = p.round(k=1, tick=True, read_index=(p.rounds % 3 == 0))
targets = [0] * G
for i, g in enumerate(range(0, G, 3)):
    targets[g] = R if i % 2 else 2
print("req", p.orc.request_leader_transfer(R - 1, targets),
      p.eng.request_leader_transfer(R - 1, targets))
for rnd in range(8):
    o, e = p.round(k=1, tick=True, read_index=(p.rounds % 3 == 0))
    print(p.rounds, "msgs", e.messages, o.messages, "fb", e.fallbacks,
          e.errors, "slow", e.elections_stepped)
    bad = 0
    for g in range(G):
        for s in range(R):
            em = by_dest(p.eng.export_outbox(g, s))
            om = by_dest(p.orc.export_outbox(g, s))
            if em != om and bad < 6:
                bad += 1
                st = p.orc.export(g, s)
                print(" g", g, "s", s, "role", st.role, "xfer", st.transfer)
                for d in sorted(set(em) | set(om)):
                    if em.get(d) != om.get(d):
                        print("   to", d, "\n    gpu", em.get(d),
                              "\n    orc", om.get(d))
    if bad:
        break

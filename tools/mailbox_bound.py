"""CPU analysis: the step pre-pass's per-follower mailbox bound against the
sends the oracle's leaders actually make, over the soak mix of
tests/test_gpu_soak.py (R = 4, forwarded proposals, ReadIndex at random
replicas, ticks, slots stopping and returning).

For every leader replica and round: the inbox (what the other replicas
sent it the round before), the pre-round state and the staged inputs give
the bound the pre-pass computes (drb_step.hpp, "mailbox: messages the round
can send to each follower s"); the round's outbox gives the sends per
follower.  Prints how often each bound passes the mailbox size while the
sends do not.  No GPU.

  python tools/mailbox_bound.py [seeds a-b] [mailbox]
"""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dragonboat_amd import abi, workload  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

M = abi.MSG


def bounds(st, inbox, R, slot, tick, staged_ri, nprops):
    """(old, new) per-follower bounds: {s: n}."""
    by = {s: [m for m in inbox if m[1] - 1 == s] for s in range(R)}
    n_rr = sum(1 for m in inbox if m[3] == M["ReplicateResp"])
    n_ri = sum(1 for m in inbox if m[3] == M["ReadIndex"])
    prop_from = sum(1 for s in range(R)
                    if any(m[3] == M["Propose"] for m in by[s]))
    adv = max(0, st.last_index - st.committed)
    nb = min(n_rr, adv)
    base_old = (staged_ri + tick + (nprops > 0) + prop_from + 2 * n_ri +
                st.ri_count + nb)
    old, new = {}, {}
    ri_from = [st.ri[i].from_ for i in range(st.ri_count)]
    for s in range(R):
        if s == slot:
            continue
        ns = len(by[s])
        nri_s = sum(1 for m in by[s] if m[3] == M["ReadIndex"])
        rr_s = sum(1 for m in by[s] if m[3] == M["ReplicateResp"])
        rej_s = any(m[3] == M["ReplicateResp"] and m[8] for m in by[s])
        prop_s = int(any(m[3] == M["Propose"] for m in by[s]))
        hb_s = ns - nri_s - rr_s - prop_s
        old[s] = base_old + ns - nri_s
        # new: a heartbeat broadcast per ReadIndex, the ReadIndexResps of
        # the queued / new requests of s only, the commit broadcasts, and
        # per ReplicateResp of s a resend only while s is paused (Wait):
        # once at the start, and again after a reject or a HeartbeatResp
        w0 = int(st.remotes[s].state != abi.REMOTE_REPLICATE)
        b = (staged_ri + tick + (nprops > 0) + prop_from + n_ri +
             sum(1 for f in ri_from if f == s + 1) + nri_s)
        b += nb + hb_s + (rr_s if rej_s else min(rr_s, w0 + hb_s))
        new[s] = b
    return old, new


def run(seed, case, mailbox, rounds=40):
    rng = random.Random(seed * 1000 + len(case))
    G, R = 48, 4
    orc = po.Cluster(G, R, seed=0x5EEDD8B0)
    orc.setup_steady(0)
    if case != "voters":
        orc.set_member_kinds(**{("nonvoting_mask" if case == "nonvoting"
                                 else "witness_mask"): 1 << 3})
    ids = [0, 1, 2, 3] + ([4] if case != "witness" else [])
    stopped = {}
    prev_out = {}  # (g, s) -> messages sent last round
    stats = dict(checks=0, old_over=0, new_over=0, sent_over=0, max_sent=0,
                 max_old=0, max_new=0, new_under=0)
    for rnd in range(rounds):
        if rnd % 8 == 3 and not stopped:
            s = rng.choice([0, 1, 2])
            gs = [g for g in range(G) if rng.random() < 0.33]
            for g in gs:
                orc.set_hosted(g, s, False)
            stopped[s] = gs
        elif rnd % 8 == 7 and stopped:
            for s, gs in stopped.items():
                for g in gs:
                    orc.set_hosted(g, s, True)
            stopped = {}
        up = [i for i in ids if i == 0 or (i - 1) not in stopped]
        k = rng.choice([0, 1, 1, 2])
        tick = rng.random() < 0.7
        read_index = rng.random() < 0.5
        ri_replica = rng.choice(up)
        prop_replica = rng.choice(up) if k else 0
        counts = None
        if k:
            counts, ents, pool = workload.build_batch(G, k, 0x5EEDD8B0, rnd,
                                                      256, 4, None)
            orc.stage_proposals(counts, k, ents, pool, prop_replica)
        if read_index:
            lo, hi = workload.build_read_index(G, 0x5EEDD8B0, rnd, rnd + 30,
                                               None)
            orc.stage_read_index(lo, hi, ri_replica)
        pre = {}
        for g in range(G):
            for s in range(R):
                st = orc.export(g, s)
                # (the export holds DRB_RI_DEPTH queued requests: a fuller
                # queue is a capacity fallback on the GPU anyway)
                if st.role == abi.LEADER and st.flags & abi.F_HOSTED and \
                        st.ri_count < abi.DRB_RI_DEPTH:
                    inbox = [m for x in range(R) if x != s
                             for m in prev_out.get((g, x), []) if m[2] == s + 1]
                    here = lambda rep: rep == 0 or rep == s + 1  # noqa: E731
                    pre[(g, s)] = bounds(
                        st, inbox, R, s, int(tick),
                        int(read_index and here(ri_replica)),
                        counts[g] if (counts and here(prop_replica)) else 0)
        orc.round(tick=tick)
        prev_out = {}
        for g in range(G):
            for s in range(R):
                prev_out[(g, s)] = orc.export_outbox(g, s)
        for (g, s), (old, new) in pre.items():
            sent = {}
            for m in prev_out[(g, s)]:
                sent[m[2] - 1] = sent.get(m[2] - 1, 0) + 1
            for f in old:
                n = sent.get(f, 0)
                stats["checks"] += 1
                stats["old_over"] += old[f] > mailbox
                stats["new_over"] += new[f] > mailbox
                stats["sent_over"] += n > mailbox
                stats["new_under"] += new[f] < n
                stats["max_sent"] = max(stats["max_sent"], n)
                stats["max_old"] = max(stats["max_old"], old[f])
                stats["max_new"] = max(stats["max_new"], new[f])
    return stats


if __name__ == "__main__":
    a, b = 11, 12
    if len(sys.argv) > 1:
        a, b = (int(x) for x in sys.argv[1].split("-"))
    mb = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    for seed in range(a, b + 1):
        for case in ("voters", "witness", "nonvoting"):
            print(seed, case, run(seed, case, mb))

// drb_lean.hpp -- the lean step kernel of listed rounds (included at the end
// of drb_step.hpp, namespace drb).
//
// In a listed round (drb_round_in.listed, C5: 4M groups, 1 % proposing,
// Quiesce) nearly every stepped replica only ticks and exchanges heartbeats:
// the leader broadcasts Heartbeat (raft.go:835-871, tick every round at
// HeartbeatRTT 1) and handles the HeartbeatResps of the last round
// (handleLeaderHeartbeatResp, raft.go:1910-1923: setActive, waitToRetry),
// a follower answers its leader's Heartbeat (handleFollowerHeartbeat ->
// handleHeartbeatMessage, raft.go:2128, 1400-1409), and both run
// node.qs (quiesce.go:40-114) and LocalTick (raft.go:571-648).  Through the
// full EXT step kernel such a round moved ~720 B per replica (counter
// traffic, profiles/pmc_c5_128.json): the whole 64 B state record read and
// written, every remote's four fields, the readIndex queue, every pre-pass
// and handler path's registers.
//
// lean_kernel<R, LEAD> takes the light part of each (role, slot) list
// (k_active_scan: no Replicate / ReplicateResp in the inbox, no staged
// proposal) and steps exactly the replicas whose round is such a heartbeat
// round -- a decision made from what it loads, before it stores anything:
//   - the group is quiet: last == committed == processed == saved_to ==
//     sm_index == applied_index, and the in-memory log holds nothing
//     (marker > last), so nothing is appended, saved, committed or applied
//     (getUpdate's entries and inMemory.appliedLogTo have nothing to do);
//   - the inbox holds only Heartbeat (follower: from its leader, a Commit
//     within its own, no ReadIndex ctx) or HeartbeatResp (leader: no ctx)
//     records at the replica's term, plus Quiesce messages;
//   - a leader has no readIndex request queued, no transfer, and every
//     remote in Replicate state at match == last (a HeartbeatResp then
//     sends no Replicate); nothing is staged for the replica;
//   - the tick triggers no election (follower) and keeps the CheckQuorum
//     quorum (leader) -- the pre-pass's ELECTION / CHECK_QUORUM tests.
// Every other replica of the light list is appended, untouched, to the
// row's escalation list (View.esc_list / esc_n), which the full step
// kernel, launched after this one, steps with the heavy part of the list
// (drb_engine.hip launch_step).  What the lean kernel does is the full
// kernel's code for these events -- the same handlers, the same quiesce
// state machine, the same record codec -- so the two are bit-identical
// for the replicas it takes; it only leaves out the loads and stores such
// a round cannot need (the readIndex queue, remote next indexes, the
// record chunks that did not change) and the code paths it cannot reach,
// so it runs at a higher occupancy.
#pragma once

namespace drb {

// waves per SIMD: the follower at 5 up to R = 3 (85 VGPRs, no spills; 6
// waves would spill 20, and at R = 5 five would spill 149), the leader at
// 4 (101 VGPRs; 5 would spill 24), where the full EXT kernels spill
// 37 / 25 VGPRs at 4 / 3 waves
// (timing variant: the round-6 first eligibility -- every entry committed,
// applied and out of memory)
#ifndef DRB_LEAN_STRICT
#define DRB_LEAN_STRICT 0
#endif
#ifndef DRB_LEAN_WHY
#define DRB_LEAN_WHY 0
#endif
#ifndef DRB_LEAN_WAVES
#define DRB_LEAN_WAVES 4
#endif
#ifndef DRB_LEAN_FOLLOW_WAVES
#define DRB_LEAN_FOLLOW_WAVES 5
#endif

template <int R, bool LEAD>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(
    LEAD || R > 3 ? DRB_LEAN_WAVES : DRB_LEAN_FOLLOW_WAVES))) void lean_kernel(
    const View v, RoundParams p) {
  const View *vp = &v;
  const BlockPos bp = block_pos(p);
  const uint32_t slot = (p.slots >> (4 * bp.y)) & 0xfu;
  const uint64_t lrow = (uint64_t)(LEAD ? 0 : 1) * v.R + slot;
  // the light part of the row's list: after its heavy lanes
  const uint64_t nh = v.act_total[2 * lrow], nl = v.act_total[2 * lrow + 1];
  const uint64_t li = (uint64_t)bp.x * blockDim.x + threadIdx.x;
  if ((uint64_t)bp.x * blockDim.x >= nl) return;  // uniform
  const uint64_t g = li < nl ? v.act_list[lrow * v.G + nh + li] : v.G;
  __shared__ RemLds<R> rl;
  __shared__ uint32_t oinfo[R * 256];
  Lane L;
  L.rl = &rl;
  L.oi = oinfo;
  L.elo = nullptr;
  L.rq = nullptr;  // (no readIndex queue: a leader with one escalates)
  L.tid = threadIdx.x;
  L.v = vp;
  L.slot = slot;
  L.g = g;
  L.round = p.round;
  L.rbuf = (uint32_t)((p.round - 1) & 1);
  L.wbuf = (uint32_t)(p.round & 1);
  L.slow = false;
  L.dirty = DRB_REM_DIRTY;
  L.members = false;
  L.peers = false;  // (lean rounds: no remote planes)
  uint32_t c_msgs = 0, c_stepped = 0;
  bool esc = false;  // escalated to the full kernel
  // records per sender a heartbeat round holds: the tick's Heartbeat, or
  // the answer to it (a second one -- a ReadIndex's -- carries a ctx and
  // escalates anyway)
  constexpr int NREC = 1;
  // Every load of the lane first, none depending on another: the flags,
  // the record, the inbox headers and -- speculatively, before the headers
  // say how many there are -- the first non-Replicate record of each
  // sender, the quiesce state and tick counter, the leader's remotes.  A
  // lane then waits for one memory round trip, where the full kernel's
  // chain of decisions waits for several.
  const bool valid = g < v.G;
  const bool qon = v.quiesce;
  uint32_t flags = 0, role = 0, fbw = 0, ric = 0, pcount = 0;
  uint4 pkq[4], meta[R], rec[R][NREC], riq = make_uint4(0, 0, 0, 0);
  uint64_t qsv[5] = {0, 0, 0, 0, 0}, tick_count = 0;
  uint64_t rmatch[R];
  uint32_t rstate[R], ractive[R];
  // (meta, rec, rmatch and rstate of the lane's own slot are never loaded
  // and never read: left undefined, so that the compiler merges the loaded
  // and the skipped path without a copy -- a copy of a loaded register
  // waits for the load, which split the follower's loads into two round
  // trips)
#pragma unroll
  for (int c = 0; c < 4; ++c) pkq[c] = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int s = 0; s < R; ++s) ractive[s] = 0;
  if (valid) {
    flags = v.u32[u32_ix(v, W_FLAGS, slot, g)];
    role = v.u32[u32_ix(v, W_ROLE, slot, g)];
    fbw = v.u32[u32_ix(v, W_FB_REASON, slot, g)];
    ric = v.u32[u32_ix(v, W_RI_COUNT, slot, g)];
#pragma unroll
    for (int c = 0; c < 4; ++c) pkq[c] = v.pk[pk_ix(v, c, slot, g)];
#pragma unroll
    for (int s = 0; s < R; ++s) {
      if ((uint32_t)s == slot) continue;
      meta[s] = v.mbox_meta[mmeta_ix(v, L.rbuf, s, slot, g)];
#pragma unroll
      for (int j = 0; j < NREC; ++j)
        rec[s][j] = v.mbox[mbox_ix(v, L.rbuf, s, slot,
                                   rec_pos(false, (uint32_t)j, v.MB), 0, g)];
    }
    if (qon) {
      qsv[0] = v.u64[u64_ix(v, F_QS_TICK, slot, g)];
      qsv[1] = v.u64[u64_ix(v, F_QS_IDLE, slot, g)];
      qsv[2] = v.u64[u64_ix(v, F_QS_SINCE, slot, g)];
      qsv[3] = v.u64[u64_ix(v, F_QS_EXIT, slot, g)];
      qsv[4] = v.u64[u64_ix(v, F_QS_BASE, slot, g)];
    }
    if (p.tick) tick_count = v.u64[u64_ix(v, F_TICK_COUNT, slot, g)];
    if (LEAD) {
#pragma unroll
      for (int s = 0; s < R; ++s) {
        if ((uint32_t)s != slot) {
          rmatch[s] = v.rem_match[rem_ix(v, slot, s, g)];
          rstate[s] = v.rem_state[rem_ix(v, slot, s, g)];
        }
        ractive[s] = v.rem_active[rem_ix(v, slot, s, g)];
      }
    }
    if (prop_here(v, p, slot, LEAD))
      pcount = v.prop_count[(uint64_t)p.prop_slot * v.G + g];
    if (ri_here(v, p, slot, LEAD))
      riq = v.ri_in[(uint64_t)p.ri_slot * v.G + g];
  }
  // (the list holds hosted replicas on the fast path of this row's role)
  bool active = valid && (flags & DRB_F_HOSTED) &&
                !(flags & (DRB_F_FALLBACK | DRB_F_ERROR)) &&
                ((role == DRB_LEADER) == LEAD);
  if (active) {
    Rep<R> r;
    // the 64 B record as load_rep decodes it
    uint32_t pw0[16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      r.pw[4 * c] = pw0[4 * c] = pkq[c].x;
      r.pw[4 * c + 1] = pw0[4 * c + 1] = pkq[c].y;
      r.pw[4 * c + 2] = pw0[4 * c + 2] = pkq[c].z;
      r.pw[4 * c + 3] = pw0[4 * c + 3] = pkq[c].w;
    }
    r.last = (uint64_t)r.pw[0] | ((uint64_t)r.pw[1] << 32);
    r.term = (uint64_t)r.pw[2] | ((uint64_t)r.pw[3] << 32);
    r.base0 = r.last;
    r.leader_id = pd_get(L, r, 1, F_LEADER_ID);
    r.election_tick = pu_get(L, r, 12, 1, F_ELECTION_TICK);
    if (LEAD) r.heartbeat_tick = pu_get(L, r, 13, 0, F_HEARTBEAT_TICK);
    r.committed = pi_get(L, r, PI_COMMITTED);
    r.processed = pi_get(L, r, PI_PROCESSED);
    r.marker = pi_get(L, r, PI_MARKER);
    r.saved_to = pi_get(L, r, PI_SAVED_TO);
    r.applied_index = pi_get(L, r, PI_APPLIED_INDEX);
    r.sm_index = pi_get(L, r, PI_SM_INDEX);
    r.ring_lo = pi_get(L, r, PI_RING_LO);
    r.ring_guard = pi_get(L, r, PI_RING_GUARD);
    r.term_start = pi_get(L, r, PI_TERM_START);
    r.sm_term = 0;
    r.kv_added = 0;
    r.applied_any = false;
    r.lid_dirty = false;
    r.flags = flags;
    r.fb = fbw;
    r.ri_count = ric;
    r.role = LEAD ? DRB_LEADER : DRB_FOLLOWER;
    r.votes = 0;
#pragma unroll
    for (int d = 0; d < DRB_RI_DEPTH; ++d) {
      r.ri_ix[d] = 0;
      r.ri_fr[d] = 0;
      r.ri_cf[d] = 0;
    }
    // nothing to save (saved_to = last) or apply (processed = committed,
    // the state machine at it), nothing staged, no queue, no transfer, the
    // role of the fast path (the pre-pass's ROLE test).  Entries may still
    // be uncommitted, or applied but held in memory: updateAppliedIndex and
    // inMemory.appliedLogTo below are all such a round does with them --
    // where appliedLogTo needs a term the cache does not give, the lane
    // escalates (log_term would read the ring)
    const uint64_t la = r.sm_index;  // applied_index after updateAppliedIndex
    const bool log_to = la > 0 && la >= r.marker && r.last >= r.marker &&
                        la <= r.last;
    bool ok = r.saved_to == r.last && r.processed == r.committed &&
              r.sm_index == r.processed && r.committed <= r.last &&
              r.applied_index <= r.sm_index &&
              (!log_to || la >= r.term_start) &&
              (!DRB_LEAN_STRICT || (r.committed == r.last &&
                                    r.applied_index == r.last &&
                                    r.marker > r.last)) &&
              r.ri_count == 0 && !(flags & (F_XFER | F_XFER_REQ)) &&
              (LEAD || role == DRB_FOLLOWER) && pcount == 0 &&
              !(riq.x | riq.y | riq.z | riq.w);
#if DRB_LEAN_WHY
    uint32_t why = 0;  // (timing variant: why a lane escalates)
    if (r.committed > r.last || r.applied_index > r.sm_index) why |= 2u;
    if (r.processed != r.committed || r.saved_to != r.last ||
        r.sm_index != r.processed)
      why |= 4u;
    if (log_to && la < r.term_start) why |= 8u;
    if (r.ri_count || (flags & (F_XFER | F_XFER_REQ)) ||
        !(LEAD || role == DRB_FOLLOWER) || pcount || (riq.x | riq.y | riq.z | riq.w))
      why |= 16u;
#define DRB_WHY(b) why |= (b)
#else
#define DRB_WHY(b) (void)0
#endif
    if (LEAD) {  // the remotes: match, state, active (next is not needed)
#pragma unroll
      for (int s = 0; s < R; ++s) {
        RemoteV x;
        x.m = (uint32_t)s != slot ? rmatch[s] : 0;
        x.n = 0;
        x.st = (uint32_t)s != slot ? rstate[s] : 0;
        x.a = ractive[s];
        if ((uint32_t)s != slot &&
            (x.m != r.last || x.st != DRB_REMOTE_REPLICATE)) {
          ok = false;
          DRB_WHY(32u);
        }
        rem_put<R>(L, s, x);
      }
      rl.dirty[L.tid] = 0;
    }
    const uint32_t flags0 = r.flags, fb0 = r.fb;
    const uint32_t tag_prev = (uint32_t)(p.round - 1);
    uint64_t qs_owed = 0;
    if (qon) {
      r.qs_tick = qsv[0];
      r.qs_idle = qsv[1];
      r.qs_since = qsv[2];
      r.qs_exit = qsv[3];
      r.qs_dirty = 0;
      // (owed ticks and the base only for a replica that may have skipped
      // rounds: quiesced and at rest, step_kernel)
      if (DRB_QS_EAGER ||
          (flags & (F_QUIESCED | F_AT_REST)) == (F_QUIESCED | F_AT_REST))
        qs_owed = p.tick_no - p.tick - qsv[4];
      r.election_tick += qs_owed;
      r.qs_tick += qs_owed;
    }
    // the inbox: heartbeats only, at the replica's term
    uint32_t nrec[R];
    uint32_t qz_from = 0, resp_from = 0, total_in = 0;
#pragma unroll
    for (int s = 0; s < R; ++s) {
      nrec[s] = 0;
      if ((uint32_t)s == slot) continue;
      const bool cur = tag_is(meta[s].x, tag_prev);
      const uint32_t info = cur ? meta[s].y : 0u;
      const uint32_t ns = mi_count(info);
      if (cur && (meta[s].x & MQ_QUIESCE)) qz_from |= 1u << s;
      if (!ns) continue;
      if (mi_nrep(info) || ((info >> MI_NRI) & 0x1fu) ||
          ((info >> MI_NRR) & 0x1fu) ||
          (info & (MI_PROP | MI_REJECT | MI_TERM_OTHER |
                   (LEAD ? MI_OFF_LEADER : MI_OFF_FOLLOWER))) ||
          ((info & MI_TERM) && hi64(meta[s]) != r.term) ||
          ns > (uint32_t)NREC || (!LEAD && (uint64_t)s + 1 != r.leader_id)) {
        ok = false;
        DRB_WHY(64u);
      }
      if (info & MI_RESP) resp_from |= 1u << s;
      total_in += ns;
      nrec[s] = ns < (uint32_t)NREC ? ns : (uint32_t)NREC;
#pragma unroll
      for (int j = 0; j < NREC; ++j)
        if ((uint32_t)j < nrec[s]) {
          const uint4 c0 = rec[s][j];
          // (a record with a second chunk carries a ReadIndex ctx; one
          // that repeats the last ctx as well)
          const uint32_t t = c0.x & 0xffu;
          if ((c0.x & (MF_HAS_C1 | MF_HINT_PREV | MF_TERM_OTHER)) ||
              t != (LEAD ? DRB_MSG_HEARTBEAT_RESP : DRB_MSG_HEARTBEAT)) {
            ok = false;
            DRB_WHY(128u);
          }
          // HeartbeatResp: a = Hint; Heartbeat: a = Commit
          if (LEAD ? (hi64(c0) != 0 || c0.y != 0) : hi64(c0) > r.committed) {
            ok = false;
            DRB_WHY(128u);
          }
        }
    }
    // the tick: no election timeout (follower), the CheckQuorum quorum
    // (leader) -- the pre-pass's tests
    const bool qtick = qon && p.tick && total_in == 0 &&
                       qs_quiet_tick(v, r, qz_from);
    if (p.tick && !qtick) {
      if (LEAD) {
        if (v.check_quorum && r.election_tick + 1 >= v.election_rtt) {
          uint32_t c = 1;
#pragma unroll
          for (int s = 0; s < R; ++s)
            if ((uint32_t)s != slot &&
                (rl.a[s][L.tid] || ((resp_from >> s) & 1)))
              c++;
          if (c < (uint32_t)(R / 2 + 1)) {
            ok = false;
            DRB_WHY(16u);
          }
        }
      } else {
        const uint64_t et = (total_in ? 0 : r.election_tick) + 1;
        if (et >= ld_f(L, r, F_RAND_TIMEOUT)) {
          ok = false;
          DRB_WHY(16u);
        }
      }
    }
#undef DRB_WHY
#if DRB_LEAN_WHY
    if (!ok && v.phase) {  // per wave: one atomic per reason
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const uint64_t m = __ballot(b ? ((why >> b) & 1u) : 1u);
        if ((threadIdx.x & 63) == __builtin_ctzll(m) && m)
          atomicAdd(&v.phase[(LEAD ? 8 : 0) + b],
                    (unsigned long long)__popcll(m));
      }
    }
#endif
    if (!ok) {
      esc = true;  // the full step kernel takes it, untouched (below)
    } else {
      c_stepped = 1;
#pragma unroll
      for (int s = 0; s < R; ++s) oinfo[s * 256 + threadIdx.x] = 0;
      r.c1mask = 0;
      r.hc.lo = r.hc.hi = 0;
      r.hc.dests = 0;
      r.nmsgs = 0;
      r.nrtr = 0;
      r.ndropped_ri = 0;
      r.ndropped_props = 0;
      r.guard_new = ~0ull;
      r.leader_update = false;
      r.oterm = false;
      r.err = false;
      r.qs_new = false;
      // handleEvents: updateAppliedIndex (node.go:1133-1137)
      r.applied_index = r.sm_index;
      st_f(L, r, F_APPLIED, r.applied_index);
      // handleReceivedMessages: every record is a non-Replicate
#pragma unroll
      for (int s = 0; s < R; ++s) {
        if ((uint32_t)s == slot) continue;
        if (qon && ((qz_from >> s) & 1)) qs_try_enter(v, r);
        const uint64_t sterm = hi64(meta[s]);
#pragma unroll
        for (int j = 0; j < NREC; ++j) {
          if ((uint32_t)j >= nrec[s]) continue;
          uint64_t plo = 0, phi = 0;
          const Msg m =
              msg_decode(rec[s][j], make_uint4(0, 0, 0, 0), sterm, plo, phi);
          if (qon) qs_record(v, r, m.type);  // (no ctx: as its type)
          if (LEAD)
            leader_heartbeat_resp(L, r, s, m);
          else
            follower_heartbeat(L, r, s, m);
        }
      }
      // LocalTick (node.tick node.go:1562 -> raft.tick raft.go:571-648)
      bool quiet = false;
      if (p.tick && qon) {
        qs_tick_once(v, r);
        quiet = qs_quiesced(r);
      }
      if (p.tick && quiet) {
        r.election_tick++;  // raft.quiescedTick (raft.go:650-656)
      } else if (p.tick) {
        over_st(L, F_TICK_COUNT, tick_count + 1);
        if (LEAD) {
          r.election_tick++;
          if (r.election_tick >= v.election_rtt) {
            r.election_tick = 0;
            if (v.check_quorum) {  // leaderHasQuorum: active flags cleared
#pragma unroll
              for (int s = 0; s < R; ++s) rl.a[s][L.tid] = 0;
              rl.dirty[L.tid] |= 0x88888888u;
            }
          }
          r.heartbeat_tick++;
          if (r.heartbeat_tick >= v.heartbeat_rtt) {
            r.heartbeat_tick = 0;
            broadcast_heartbeat_hint(L, r, 0, 0);  // (no queued ctx)
          }
        } else {
          r.election_tick++;
        }
      }
      // stepNode: sendEnterQuiesceMessages (node.go:993-1005, 1148-1150)
      uint32_t qz_out = 0;
      if (qon && r.qs_new) {
        qz_out = ((1u << R) - 1u) & ~(1u << slot);
        r.nmsgs += R - 1;
      }
      // getUpdate (node.go:1025): no entries to save or apply, the state
      // as before unless the vote changed -- Peer.prevState, in place
      const uint64_t vote = ld_f(L, r, F_VOTE);
      const uint64_t prev_term = ld_f(L, r, F_PREV_TERM);
      const uint64_t prev_vote = ld_f(L, r, F_PREV_VOTE);
      const uint64_t prev_commit = ld_f(L, r, F_PREV_COMMIT);
      const uint64_t confirmed_index = ld_f(L, r, F_CONFIRMED_INDEX);
      const bool state_changed = !(r.term == prev_term && vote == prev_vote &&
                                   r.committed == prev_commit);
      const bool state_empty = r.term == 0 && vote == 0 && r.committed == 0;
      const bool has_update =
          r.leader_update || r.nmsgs > 0 || (!state_empty && state_changed);
      if (has_update || confirmed_index != r.applied_index) {
        if (state_changed && !state_empty) {
          if (prev_term != r.term) st_f(L, r, F_PREV_TERM, r.term);
          if (prev_vote != vote) st_f(L, r, F_PREV_VOTE, vote);
          st_f(L, r, F_PREV_COMMIT, r.committed);
        }
        if (confirmed_index != r.applied_index)
          st_f(L, r, F_CONFIRMED_INDEX, r.applied_index);
        // Peer.Commit -> entryLog.commitUpdate: nothing saved or applied;
        // inMemory.appliedLogTo (inmemory.go:138-164) as the step kernel
        // runs it, the term from the cache (la >= term_start, above)
        if (log_to) {
          st_f(L, r, F_APPLIED_TO_INDEX, la);
          st_f(L, r, F_APPLIED_TO_TERM, r.term);
          r.marker = la + 1;
        }
      }
      r.ring_guard = r.guard_new;
      // at rest (see step_kernel), and the quiesce state; nothing saved
      r.flags |= F_AT_REST;
      if (p.encode_saves) r.flags |= F_SAVE_ZERO;
      if (qon) {
        r.flags = qs_quiesced(r) ? (r.flags | F_QUIESCED)
                                 : (r.flags & ~F_QUIESCED);
        over_st(L, F_QS_TICK, r.qs_tick);
        const uint32_t qd = DRB_QS_DIRTY ? r.qs_dirty : 7u;
        if (qd & 1u) over_st(L, F_QS_IDLE, r.qs_idle);
        if (qd & 2u) over_st(L, F_QS_SINCE, r.qs_since);
        if (qd & 4u) over_st(L, F_QS_EXIT, r.qs_exit);
        if (DRB_QS_EAGER || (r.flags & F_QUIESCED))
          over_st(L, F_QS_BASE, p.tick_no);
      }
      // store_rep's record, re-based as it does (last did not move), and
      // only the 16 B chunks that changed
      const uint64_t base = r.last;
#pragma unroll
      for (int i = PI_APPLIED; i < NUM_PI; ++i) {
        const uint32_t c = pk_half(r.pw, 4 + i / 2, i & 1);
        if (c != PK_ESC16)
          pi_put(L, r, i, pk_idx_value(c, r.base0, false), base);
      }
      pi_put(L, r, PI_COMMITTED, r.committed, base);
      pi_put(L, r, PI_PROCESSED, r.processed, base);
      pi_put(L, r, PI_MARKER, r.marker, base);
      pi_put(L, r, PI_SAVED_TO, r.saved_to, base);
      pi_put(L, r, PI_SM_INDEX, r.sm_index, base);
      pi_put(L, r, PI_APPLIED_INDEX, r.applied_index, base);
      pi_put(L, r, PI_RING_LO, r.ring_lo, base);
      pi_put(L, r, PI_RING_GUARD, r.ring_guard, base);
      pi_put(L, r, PI_TERM_START, r.term_start, base);
      if (r.lid_dirty) pd_put(L, r, 1, F_LEADER_ID, r.leader_id);
      pu_put(L, r, 12, 1, F_ELECTION_TICK, r.election_tick);
      if (LEAD) pu_put(L, r, 13, 0, F_HEARTBEAT_TICK, r.heartbeat_tick);
      r.pw[0] = (uint32_t)r.last;
      r.pw[1] = (uint32_t)(r.last >> 32);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (r.pw[4 * c] != pw0[4 * c] || r.pw[4 * c + 1] != pw0[4 * c + 1] ||
            r.pw[4 * c + 2] != pw0[4 * c + 2] ||
            r.pw[4 * c + 3] != pw0[4 * c + 3])
          v.pk[pk_ix(v, c, slot, g)] =
              make_uint4(r.pw[4 * c], r.pw[4 * c + 1], r.pw[4 * c + 2],
                         r.pw[4 * c + 3]);
      if (r.flags != flags0) v.u32[u32_ix(v, W_FLAGS, slot, g)] = r.flags;
      if (r.fb != fb0) v.u32[u32_ix(v, W_FB_REASON, slot, g)] = r.fb;
      if (LEAD) {  // the remote fields that changed (active flags)
        const uint32_t dm = rl.dirty[L.tid];
#pragma unroll
        for (int s = 0; s < R; ++s)
          if ((dm >> (4 * s)) & 8u)
            v.rem_active[rem_ix(v, slot, s, g)] = rl.a[s][L.tid];
      }
      c_msgs = r.nmsgs;
      // outbox headers of the destinations that got records (step_kernel)
#pragma unroll
      for (int s = 0; s < R; ++s) {
        const uint32_t w = oinfo[s * 256 + threadIdx.x];
        const bool qz = (qz_out >> s) & 1u;
        if (mi_count(w) || qz) {
          uint4 meta = mk4(0, r.term);
          meta.x = ((uint32_t)p.round & MQ_TAG) | (qz ? MQ_QUIESCE : 0u);
          meta.y = w;
          v.mbox_meta[mmeta_ix(v, L.wbuf, slot, (uint32_t)s, g)] = meta;
          ((uint8_t *)&v.inbox_tag[((uint64_t)L.wbuf * v.R + s) * v.G + g])
              [slot] = tag_byte(p.round, w);
        }
      }
      // (a replica that ended its last round at rest left no ReadyToRead)
      if (DRB_QS_EAGER || !(flags0 & F_AT_REST))
        v.rtr_count[ix(v, slot, g)] = 0;
      if (p.encode_saves && (DRB_QS_EAGER || !(flags0 & F_SAVE_ZERO)))
        v.save_len[ix(v, slot, g)] = 0;
    }
  }
  // the escalated lanes onto the row's list: one atomic per wave, into
  // the list segment of this block (block index mod ESC_SPLIT; global
  // atomics on one address serialise, ~14 ns each)
  {
    const uint64_t bal = __ballot(esc);
    if (bal) {
      const uint32_t lane = threadIdx.x & 63u;
      const uint32_t first = (uint32_t)__ffsll((long long)bal) - 1u;
      const uint32_t k = bp.x % ESC_SPLIT;
      const uint64_t seg = esc_seg(v.G);
      unsigned base = 0;
      if (lane == first)
        base = atomicAdd(&v.esc_n[lrow * ESC_SPLIT + k],
                         (unsigned)__popcll(bal));
      base = (unsigned)__shfl((int)base, (int)first, 64);
      if (esc)
        v.esc_list[(lrow * ESC_SPLIT + k) * seg + base +
                   (unsigned)__popcll(bal & ((1ull << lane) - 1ull))] =
            (uint32_t)g;
    }
  }
  uint32_t cnt[NUM_COUNTERS] = {};
  cnt[C_MESSAGES] = c_msgs;
  cnt[C_STEPPED] = c_stepped;
  cnt[C_LEAN] = c_stepped;
  block_counters<LEAD, 0, NUM_COUNTERS>(v, slot, bp, cnt);
}

}  // namespace drb

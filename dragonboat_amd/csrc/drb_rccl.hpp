// drb_rccl.hpp -- the cross-rank mailbox exchange of a process-per-GPU host
// inside the C ABI (drb_exchange_plan / drb_exchange_rccl /
// drb_exchange_rccl_roles, include/drb_engine.h), included at the end of
// drb_engine.hip.
//
// Replaces Transport.Send -> handleRequest (internal/transport/
// transport.go:346, :305) for GPU-resident replicas spread over ranks
// (SURVEY 8e, C4): after a round, every remote plane that can carry
// fast-path messages moves at its full capacity (full_word: what the step
// pre-pass bounds), so no counts are read and nothing waits on the host.
// The operations are the same list dragonboat_amd/exchange.py builds for
// torch.distributed (plan(), fixed mode); here they go straight to RCCL's
// point-to-point calls in one group on the engine stream, so a Go host
// (cgo) needs no Python and no torch.
#pragma once

#include <rccl/rccl.h>

// the leader slots whose planes move (leader_mask), as every rank computes
// them: plane (a, b) when a or b is a leader slot on some rank, every
// remote plane with elections
static void xplan_words(const drb_engine *e, uint32_t leader_mask,
                        std::vector<uint32_t> *row) {
  const View &v = e->v;
  const uint32_t R = v.R;
  row->assign(R * R, 0u);
  for (uint32_t a = 0; a < R; ++a)
    for (uint32_t b = 0; b < R; ++b)
      if (a != b &&
          ((((leader_mask >> a) | (leader_mask >> b)) & 1u) || v.elections))
        (*row)[a * R + b] = full_word(v, (leader_mask >> a) & 1u);
}

// the transfers of one exchange step from every rank's plane words
// (words[q * R * R + a * R + b]: rank q's word of plane (a, b)): this rank
// sends plane (a, b) at its own word and receives it at its sender's, in
// the same (from, to, region) order on every rank
static int xplan_ops(drb_engine *e, const uint32_t *words, drb_xfer *ops,
                     size_t cap, size_t *n_ops) {
  *n_ops = 0;
  const View &v = e->v;
  const uint32_t R = v.R;
  if (v.place_world < 2) return DRB_OK;
  size_t n = 0;
  auto put = [&](uint32_t peer, uint32_t recv, const drb_region &r) {
    if (n < cap) ops[n] = drb_xfer{peer, recv, r.ptr, r.bytes};
    ++n;
  };
  drb_region reg[DRB_PLANE_REGIONS];
  for (uint32_t a = 0; a < R; ++a)
    for (uint32_t b = 0; b < R; ++b) {
      if (a == b) continue;
      const int dst = drb_place_peer(v.place_world, v.place_rank, a, b, 0);
      if (dst < 0) continue;
      const int src = drb_place_peer(v.place_world, v.place_rank, a, b, 1);
      const uint32_t ws = words[(uint64_t)v.place_rank * R * R + a * R + b];
      const uint32_t wr = words[(uint64_t)src * R * R + a * R + b];
      if (ws) {
        const int k = drb_plane_regions(e, a, b, ws, 0, reg);
        if (k < 0) return k;
        for (int i = 0; i < k; ++i) put((uint32_t)dst, 0, reg[i]);
      }
      if (wr) {
        const int k = drb_plane_regions(e, a, b, wr, 1, reg);
        if (k < 0) return k;
        for (int i = 0; i < k; ++i) put((uint32_t)src, 1, reg[i]);
      }
    }
  *n_ops = n;
  return n > cap && ops ? DRB_ERANGE : DRB_OK;
}

extern "C" int drb_exchange_plan(drb_engine *e, uint32_t leader_mask,
                                 drb_xfer *ops, size_t cap, size_t *n_ops) {
  if (!e || !n_ops || (cap && !ops)) return DRB_EINVAL;
  *n_ops = 0;
  const View &v = e->v;
  if (v.place_world < 2) return DRB_OK;
  // the fixed step: the same full-capacity row on every rank
  std::vector<uint32_t> row, all;
  xplan_words(e, leader_mask, &row);
  for (uint32_t q = 0; q < v.place_world; ++q)
    all.insert(all.end(), row.begin(), row.end());
  return xplan_ops(e, all.data(), ops, cap, n_ops);
}

extern "C" int drb_exchange_plan_words(drb_engine *e, const uint32_t *words,
                                       drb_xfer *ops, size_t cap,
                                       size_t *n_ops) {
  if (!e || !words || !n_ops || (cap && !ops)) return DRB_EINVAL;
  return xplan_ops(e, words, ops, cap, n_ops);
}

// the transfers as ncclSend / ncclRecv in one group on the engine stream
static int xpost_rccl(drb_engine *e, ncclComm_t c,
                      const std::vector<drb_xfer> &ops) {
  bool ok = ncclGroupStart() == ncclSuccess;
  for (size_t i = 0; ok && i < ops.size(); ++i) {
    const drb_xfer &x = ops[i];
    ok = (x.recv ? ncclRecv(x.ptr, x.bytes, ncclUint8, (int)x.peer, c,
                            e->stream)
                 : ncclSend(x.ptr, x.bytes, ncclUint8, (int)x.peer, c,
                            e->stream)) == ncclSuccess;
  }
  ok = (ncclGroupEnd() == ncclSuccess) && ok;
  if (!ok) return DRB_EDEVICE;
  for (const drb_xfer &x : ops)
    if (x.recv) e->xcopy_bytes += x.bytes;  // (drb_exchange_bytes: inbound)
  return DRB_OK;
}

// comm must be the placement's: rank place_rank of place_world
static int xcomm_check(const drb_engine *e, ncclComm_t c) {
  int nranks = 0, me = -1;
  if (ncclCommCount(c, &nranks) != ncclSuccess ||
      ncclCommUserRank(c, &me) != ncclSuccess)
    return DRB_EDEVICE;
  if ((uint32_t)nranks != e->v.place_world ||
      (uint32_t)me != e->v.place_rank)
    return DRB_EINVAL;
  return DRB_OK;
}

extern "C" int drb_exchange_rccl_counted(drb_engine *e, void *comm) {
  if (!e || !comm) return DRB_EINVAL;
  if (!e->bound.empty()) return DRB_EINVAL;  // (drb_exchange_local_bind)
  if (e->v.place_world < 2) return drb_exchange_mark(e);
  ncclComm_t c = (ncclComm_t)comm;
  if (int rc = xcomm_check(e, c)) return rc;
  const uint32_t R = e->v.R, W = e->v.place_world;
  const size_t rr = (size_t)R * R;
  // this rank's words (a synchronisation of the engine stream), then every
  // rank's (an all-gather on the engine stream, read back)
  std::vector<uint32_t> mine(rr), all(rr * W);
  if (int rc = drb_plane_counts(e, mine.data())) return rc;
  void *d = nullptr;
  if (scratch(e, 4 * rr * (W + 1), &d)) return DRB_ENOMEM;
  uint32_t *dm = (uint32_t *)d, *da = dm + rr;
  HIPCHK(hipSetDevice(e->cfg.device));
  HIPCHK(hipMemcpyAsync(dm, mine.data(), 4 * rr, hipMemcpyHostToDevice,
                        e->stream));
  if (ncclAllGather(dm, da, rr, ncclUint32, c, e->stream) != ncclSuccess)
    return DRB_EDEVICE;
  HIPCHK(hipMemcpyAsync(all.data(), da, 4 * rr * W, hipMemcpyDeviceToHost,
                        e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  size_t n = 0;
  if (int rc = xplan_ops(e, all.data(), nullptr, 0, &n)) return rc;
  std::vector<drb_xfer> ops(n);
  if (int rc = xplan_ops(e, all.data(), ops.data(), n, &n)) return rc;
  if (int rc = xpost_rccl(e, c, ops)) return rc;
  return drb_exchange_mark(e);
}

extern "C" int drb_exchange_rccl(drb_engine *e, void *comm,
                                 uint32_t leader_mask) {
  if (!e || !comm) return DRB_EINVAL;
  if (!e->bound.empty()) return DRB_EINVAL;  // (drb_exchange_local_bind)
  if (e->v.place_world < 2) return drb_exchange_mark(e);
  ncclComm_t c = (ncclComm_t)comm;
  if (int rc = xcomm_check(e, c)) return rc;
  size_t n = 0;
  if (int rc = drb_exchange_plan(e, leader_mask, nullptr, 0, &n)) return rc;
  std::vector<drb_xfer> ops(n);
  if (int rc = drb_exchange_plan(e, leader_mask, ops.data(), n, &n)) return rc;
  HIPCHK(hipSetDevice(e->cfg.device));
  // one group on the engine stream: RCCL's kernels run behind the round
  // that wrote the outbox planes, and the next round behind them
  if (int rc = xpost_rccl(e, c, ops)) return rc;
  return drb_exchange_mark(e);
}

extern "C" int drb_exchange_rccl_roles(drb_engine *e, void *comm,
                                       uint32_t *leader_mask) {
  if (!e || !comm || !leader_mask) return DRB_EINVAL;
  // the OR over the ranks as a max over one byte per slot
  const uint32_t R = e->v.R;
  uint8_t host[32] = {0};
  for (uint32_t s = 0; s < R; ++s) host[s] = (e->role_slots[0] >> s) & 1u;
  void *d = nullptr;
  if (scratch(e, 32, &d)) return DRB_ENOMEM;
  HIPCHK(hipSetDevice(e->cfg.device));
  HIPCHK(hipMemcpyAsync(d, host, 32, hipMemcpyHostToDevice, e->stream));
  if (ncclAllReduce(d, d, R, ncclUint8, ncclMax, (ncclComm_t)comm,
                    e->stream) != ncclSuccess)
    return DRB_EDEVICE;
  HIPCHK(hipMemcpyAsync(host, d, 32, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  uint32_t m = 0;
  for (uint32_t s = 0; s < R; ++s) m |= (host[s] ? 1u : 0u) << s;
  *leader_mask = m;
  return DRB_OK;
}

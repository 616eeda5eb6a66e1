// drb_hsa.hpp -- the engine's own SDMA transfers between pinned host
// memory and HBM (hsa_amd_memory_async_copy_on_engine), included by
// drb_engine.hip.
//
// HIP picks the copy engine of a hipMemcpyAsync itself: inside a PyTorch
// process a D2H ran as blit kernels that took CUs from the round, or on one
// SDMA queue at ~29 GB/s, and an upload and a download that landed on the
// same engine ran one after the other (tools/calib_d2h, tools/calib_sdma,
// profiles/r05_worker).  The step-worker loop's two big transfers -- the
// staged proposals up (drb_stage_proposals_packed*) and the round's
// outputs down (drb_worker_export) -- therefore go to two different fast
// engines of the engine's choosing: each moves ~56 GB/s (PCIe-bound; one
// engine per direction is enough), takes no CU, and neither waits for the
// other.
#pragma once

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

struct HsaXfer {
  int state = 0;  // 0: not tried, 1: ready, -1: unavailable (HIP copies)
  hsa_agent_t cpu{}, gpu{};
  uint32_t up = 0, down = 0;  // the engines (hsa_amd_sdma_engine_id_t)
  hsa_signal_t up_done{0};    // the staged upload's copies outstanding
};

// the HSA agents of HIP device `device` and of host memory, and the two
// engines: of the fast ones (0-3 move 56 GB/s, 4-15 7-13 GB/s), the
// preferred first
static bool hsa_xfer_init(int device, HsaXfer *x) {
  if (x->state) return x->state > 0;
  x->state = -1;
  int bus = -1, dev = -1, dom = -1;
  if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) !=
          hipSuccess ||
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) !=
          hipSuccess ||
      hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device) !=
          hipSuccess)
    return false;
  if (hsa_init() != HSA_STATUS_SUCCESS) return false;
  struct Find {
    int bus, dev, dom;
    bool cpu_ok, gpu_ok;
    hsa_agent_t cpu, gpu;
  } f{bus, dev, dom, false, false, {}, {}};
  (void)hsa_iterate_agents(
      [](hsa_agent_t a, void *p) {
        Find &f = *(Find *)p;
        hsa_device_type_t t;
        if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) !=
            HSA_STATUS_SUCCESS)
          return HSA_STATUS_SUCCESS;
        if (t == HSA_DEVICE_TYPE_CPU && !f.cpu_ok) {
          f.cpu = a;
          f.cpu_ok = true;
        } else if (t == HSA_DEVICE_TYPE_GPU && !f.gpu_ok) {
          uint32_t bdf = 0, dom = 0;
          (void)hsa_agent_get_info(
              a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
          (void)hsa_agent_get_info(
              a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
          if ((int)(bdf >> 8) == f.bus && (int)((bdf >> 3) & 31) == f.dev &&
              (int)dom == f.dom) {
            f.gpu = a;
            f.gpu_ok = true;
          }
        }
        return HSA_STATUS_SUCCESS;
      },
      &f);
  uint32_t avail = 0, pref = 0;
  if (!f.cpu_ok || !f.gpu_ok ||
      hsa_amd_memory_copy_engine_status(f.cpu, f.gpu, &avail) !=
          HSA_STATUS_SUCCESS ||
      !avail ||
      hsa_signal_create(0, 0, nullptr, &x->up_done) != HSA_STATUS_SUCCESS) {
    (void)hsa_shut_down();
    return false;
  }
  (void)hsa_amd_memory_get_preferred_copy_engine(f.cpu, f.gpu, &pref);
  const uint32_t m = (avail & 0xfu) ? (avail & 0xfu) : avail;
  uint32_t cand[2] = {0, 0};
  int n = 0;
  for (int pass = 0; pass < 2; ++pass)
    for (int b = 0; b < 16 && n < 2; ++b) {
      const uint32_t bit = 1u << b;
      if ((m & bit) && (((pref & bit) != 0) == (pass == 0))) cand[n++] = bit;
    }
  x->cpu = f.cpu;
  x->gpu = f.gpu;
  x->up = cand[0];
  x->down = n > 1 ? cand[1] : cand[0];
  x->state = 1;
  if (getenv("DRB_XFER_LOG"))
    fprintf(stderr, "drb: SDMA engines available 0x%x preferred 0x%x; up "
            "0x%x, down 0x%x\n", avail, pref, x->up, x->down);
  return true;
}

static void hsa_xfer_fini(HsaXfer *x) {
  if (x->state > 0) {
    (void)hsa_signal_destroy(x->up_done);
    (void)hsa_shut_down();
  }
  x->state = 0;
}

// until signal s drops below 1
static void hsa_wait_zero(hsa_signal_t s) {
  while (hsa_signal_wait_scacquire(s, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                   HSA_WAIT_STATE_BLOCKED) >= 1) {
  }
}

// host memory the GPU agent can read directly (pinned by HIP)
static bool hsa_host_pinned(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

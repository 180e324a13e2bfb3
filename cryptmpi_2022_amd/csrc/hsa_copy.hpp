// hsa_copy.hpp — device-to-host copies on an SDMA engine for the host pipeline (cmpi_aead.hip,
// output mode 4).  hipMemcpyAsync D2H into page-locked memory runs as a blit kernel
// (__amd_rocclr_copyBuffer), and while one runs no other command of the pipeline starts — not the
// next chunk's kernel, not the next input copy on the copy engine — so each chunk paid kernel +
// D2H in series (rocprofv3 --kernel-trace --memory-copy-trace, profiles/r06_hostpath_timelines.txt).
// hsa_amd_memory_async_copy between the GPU agent and a CPU agent runs on an SDMA engine beside
// the kernels; its completion is an HSA signal the host waits on.
#pragma once
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

namespace {

struct HsaAgents {
  bool ok = false;
  hsa_agent_t gpu{}, cpu{};
  uint32_t eng_h2d = 0, eng_d2h = 0;  // SDMA engine ids (hsa_amd_sdma_engine_id_t), 0 = the runtime's choice
};

struct AgentFind {
  uint32_t bdf = 0, domain = 0;
  HsaAgents* out = nullptr;
  bool have_gpu = false, have_cpu = false;
};

hsa_status_t find_agent(hsa_agent_t a, void* p) {
  AgentFind& f = *static_cast<AgentFind*>(p);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_CPU && !f.have_cpu) {
    f.out->cpu = a;
    f.have_cpu = true;
  } else if (t == HSA_DEVICE_TYPE_GPU && !f.have_gpu) {
    uint32_t bdf = 0, dom = 0;
    if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) == HSA_STATUS_SUCCESS &&
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom) == HSA_STATUS_SUCCESS &&
        bdf == f.bdf && dom == f.domain) {
      f.out->gpu = a;
      f.have_gpu = true;
    }
  }
  return HSA_STATUS_SUCCESS;
}

// The HSA agents of HIP device `dev` (matched by PCI domain / bus / device) and a CPU agent, once
// per device; ok = false when any is missing (the caller then keeps hipMemcpyAsync).
const HsaAgents& hsa_agents(int dev) {
  static HsaAgents tab[16];
  static std::once_flag once[16];
  if (dev < 0 || dev >= 16) {
    static const HsaAgents none;
    return none;
  }
  std::call_once(once[dev], [dev] {
    int bus = 0, d = 0, dom = 0;
    if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, dev) != hipSuccess ||
        hipDeviceGetAttribute(&d, hipDeviceAttributePciDeviceId, dev) != hipSuccess ||
        hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, dev) != hipSuccess)
      return;
    if (hsa_init() != HSA_STATUS_SUCCESS) return;  // reference-counted: HIP has initialised the runtime
    AgentFind f;
    f.bdf = ((uint32_t)bus << 8) | ((uint32_t)d << 3);
    f.domain = (uint32_t)dom;
    f.out = &tab[dev];
    (void)hsa_iterate_agents(find_agent, &f);
    tab[dev].ok = f.have_gpu && f.have_cpu;
    // one engine per direction when the runtime names preferred engines (on the MI355X it names
    // none: the runtime's own choice then, measured equal to fixed engines; CMPI_SDMA_ENGINES=0
    // never picks)
    const char* env = getenv("CMPI_SDMA_ENGINES");
    uint32_t mh = 0, md = 0;
    if (tab[dev].ok && !(env && atoi(env) == 0) &&
        hsa_amd_memory_get_preferred_copy_engine(tab[dev].gpu, tab[dev].cpu, &mh) == HSA_STATUS_SUCCESS &&
        hsa_amd_memory_get_preferred_copy_engine(tab[dev].cpu, tab[dev].gpu, &md) == HSA_STATUS_SUCCESS && mh && md) {
      const uint32_t h = mh & (~mh + 1u);
      const uint32_t rest = md & ~h;
      tab[dev].eng_h2d = h;
      tab[dev].eng_d2h = rest ? (rest & (~rest + 1u)) : (md & (~md + 1u));
    }
  });
  return tab[dev];
}

// Wait until the signal is at most 0 (its copies done; < 0: one failed) and return its value.
// hsa_signal_wait_* may return before the condition holds, so the observed value is checked: a
// copy still in flight when the call returned wrote into staging the next allocation reused
// (round 6: an illegal address in a later test, before this loop).
hsa_signal_value_t sig_wait_done(hsa_signal_t sg) {
  hsa_signal_value_t v;
  while ((v = hsa_signal_wait_scacquire(sg, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE)) > 0) {
  }
  return v;
}

// An SDMA copy on `eng` (0: the runtime picks the engine).
hsa_status_t sdma_copy(void* dst, hsa_agent_t da, const void* src, hsa_agent_t sa, size_t n, uint32_t ndep,
                       const hsa_signal_t* deps, hsa_signal_t done, uint32_t eng) {
  if (!eng) return hsa_amd_memory_async_copy(dst, da, src, sa, n, ndep, deps, done);
  return hsa_amd_memory_async_copy_on_engine(dst, da, src, sa, n, ndep, deps, done, (hsa_amd_sdma_engine_id_t)eng, false);
}

}  // namespace

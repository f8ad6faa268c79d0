// hsa_probe.hip -- launch-to-return latency of a one-workgroup kernel that
// publishes its completion in pinned host memory (the shape of the library's
// small synchronous calls), launched (a) through hipLaunchKernel and (b) as an
// AQL packet written by this thread into its own HSA queue.  The kernel object
// for (b) is the one HIP loaded for (a), found through the loader extension
// (hsa_ven_amd_loader_iterate_executables) -- no second code object.
//
// Times per call, medians over interleaved rounds: host enqueue alone, and
// enqueue -> flag seen by the host (spin), and for (b) also the packet's
// completion signal waited on instead of the flag.
//
// build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/hsa_probe.hip -lhsa-runtime64 -o tools/hsa_probe.exe
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)
#define HK(x)                                                                                  \
    do {                                                                                       \
        hsa_status_t s_ = (x);                                                                 \
        if (s_ != HSA_STATUS_SUCCESS) {                                                        \
            const char* m_ = nullptr;                                                          \
            hsa_status_string(s_, &m_);                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, m_ ? m_ : "?");          \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

struct FlagArgs {
    uint32_t* flag;
    uint32_t seq;
    uint32_t pad;
};

extern "C" __global__ void __launch_bounds__(64) zfec_probe_flag(FlagArgs a) {
    if (threadIdx.x == 0) __hip_atomic_store(a.flag, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Find {
    const char* name;
    hsa_agent_t agent;
    uint64_t kobj = 0;
    uint32_t kernarg = 0, group = 0, priv = 0;
};

static hsa_status_t on_symbol(hsa_executable_t, hsa_agent_t, hsa_executable_symbol_t sym, void* data) {
    Find* f = static_cast<Find*>(data);
    hsa_symbol_kind_t kind;
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &kind));
    if (kind != HSA_SYMBOL_KIND_KERNEL) return HSA_STATUS_SUCCESS;
    uint32_t len = 0;
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &len));
    std::string n(len, '\0');
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_NAME, &n[0]));
    if (n != std::string(f->name) + ".kd" && n != f->name) return HSA_STATUS_SUCCESS;
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &f->kobj));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &f->kernarg));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &f->group));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &f->priv));
    return HSA_STATUS_INFO_BREAK;
}

static hsa_status_t on_exe(hsa_executable_t exe, void* data) {
    Find* f = static_cast<Find*>(data);
    hsa_status_t s = hsa_executable_iterate_agent_symbols(exe, f->agent, on_symbol, data);
    return s == HSA_STATUS_INFO_BREAK ? s : HSA_STATUS_SUCCESS;
}

static hsa_status_t on_agent(hsa_agent_t a, void* data) {
    hsa_device_type_t t;
    HK(hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t));
    auto* v = static_cast<std::vector<hsa_agent_t>*>(data);
    if (t == HSA_DEVICE_TYPE_GPU) v[0].push_back(a);
    if (t == HSA_DEVICE_TYPE_CPU) v[1].push_back(a);
    return HSA_STATUS_SUCCESS;
}

static hsa_status_t on_pool(hsa_amd_memory_pool_t p, void* data) {
    hsa_amd_segment_t seg;
    HK(hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg));
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    uint32_t fl = 0;
    HK(hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl));
    if (fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) {
        *static_cast<hsa_amd_memory_pool_t*>(data) = p;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 2000;
    CK(hipSetDevice(0));
    CK(hipFree(nullptr));
    uint32_t* flag = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&flag), 64, hipHostMallocDefault));
    uint32_t* flag_dev = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&flag_dev), flag, 0));
    *flag = 0;
    uint32_t seq = 0;
    // (a) once through HIP, so HIP has loaded the code object
    FlagArgs a{flag_dev, ++seq, 0};
    hipLaunchKernelGGL(zfec_probe_flag, dim3(1), dim3(64), 0, 0, a);
    CK(hipDeviceSynchronize());
    if (*flag != seq) {
        fprintf(stderr, "flag not written\n");
        return 1;
    }

    HK(hsa_init());
    std::vector<hsa_agent_t> agents[2];
    HK(hsa_iterate_agents(on_agent, agents));
    if (agents[0].empty() || agents[1].empty()) {
        fprintf(stderr, "no GPU / CPU agent\n");
        return 1;
    }
    int hip_pci_bus = 0, hip_pci_dev = 0, hip_pci_dom = 0;
    CK(hipDeviceGetAttribute(&hip_pci_bus, hipDeviceAttributePciBusId, 0));
    CK(hipDeviceGetAttribute(&hip_pci_dev, hipDeviceAttributePciDeviceId, 0));
    CK(hipDeviceGetAttribute(&hip_pci_dom, hipDeviceAttributePciDomainID, 0));
    hsa_agent_t gpu = agents[0][0];
    for (hsa_agent_t g : agents[0]) {
        uint32_t bdf = 0, dom = 0;
        HK(hsa_agent_get_info(g, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf));
        HK(hsa_agent_get_info(g, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &dom));
        if (int(bdf >> 8) == hip_pci_bus && int((bdf >> 3) & 31) == hip_pci_dev && int(dom) == hip_pci_dom) gpu = g;
    }
    printf("gpu agents %zu, pci %04x:%02x:%02x\n", agents[0].size(), hip_pci_dom, hip_pci_bus, hip_pci_dev);

    Find f{"zfec_probe_flag", gpu};
    hsa_ven_amd_loader_1_03_pfn_t loader{};
    HK(hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof loader, &loader));
    HK(loader.hsa_ven_amd_loader_iterate_executables(on_exe, &f) == HSA_STATUS_INFO_BREAK ? HSA_STATUS_SUCCESS
                                                                                          : HSA_STATUS_ERROR);
    printf("kernel object %#lx kernarg %u group %u private %u\n", (unsigned long)f.kobj, f.kernarg, f.group, f.priv);
    if (!f.kobj) return 1;

    hsa_queue_t* q = nullptr;
    HK(hsa_queue_create(gpu, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
    hsa_amd_memory_pool_t kpool{};
    HK(hsa_amd_agent_iterate_memory_pools(agents[1][0], on_pool, &kpool) == HSA_STATUS_INFO_BREAK
           ? HSA_STATUS_SUCCESS
           : HSA_STATUS_ERROR);
    void* karg = nullptr;
    const size_t kbytes = std::max<size_t>(f.kernarg, 256);
    HK(hsa_amd_memory_pool_allocate(kpool, kbytes, 0, &karg));
    HK(hsa_amd_agents_allow_access(1, &gpu, nullptr, karg));
    memset(karg, 0, kbytes);
    hsa_signal_t done;
    HK(hsa_signal_create(1, 0, nullptr, &done));

    auto dispatch = [&](uint32_t s, bool with_signal) {
        FlagArgs* ka = static_cast<FlagArgs*>(karg);
        ka->flag = flag_dev;
        ka->seq = s;
        // hidden arguments (code object v5): block counts and group sizes
        char* hidden = static_cast<char*>(karg) + 16;
        const uint32_t bc[3] = {1, 1, 1};
        const uint16_t gs[3] = {64, 1, 1};
        memcpy(hidden, bc, sizeof bc);
        memcpy(hidden + 12, gs, sizeof gs);
        const uint16_t dims = 1;
        memcpy(hidden + 64, &dims, 2);
        if (with_signal) hsa_signal_store_relaxed(done, 1);
        const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
        while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {
        }
        auto* pk = static_cast<hsa_kernel_dispatch_packet_t*>(q->base_address) + (idx & (q->size - 1));
        pk->workgroup_size_x = 64;
        pk->workgroup_size_y = 1;
        pk->workgroup_size_z = 1;
        pk->grid_size_x = 64;
        pk->grid_size_y = 1;
        pk->grid_size_z = 1;
        pk->private_segment_size = f.priv;
        pk->group_segment_size = f.group;
        pk->kernel_object = f.kobj;
        pk->kernarg_address = karg;
        pk->reserved2 = 0;
        pk->completion_signal = with_signal ? done : hsa_signal_t{0};
        const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                (1 << HSA_PACKET_HEADER_BARRIER) |
                                (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
        const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
        __atomic_store_n(reinterpret_cast<uint32_t*>(pk), header | (uint32_t(setup) << 16), __ATOMIC_RELEASE);
        hsa_signal_store_screlease(q->doorbell_signal, idx);
    };
    auto spin = [&](uint32_t s) {
        const double t0 = now_us();
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != s) {
            if (now_us() - t0 > 1e6) {
                fprintf(stderr, "flag timeout\n");
                exit(1);
            }
        }
    };

    // one HSA dispatch checked before timing
    dispatch(++seq, true);
    if (hsa_signal_wait_scacquire(done, HSA_SIGNAL_CONDITION_LT, 1, 1000000000ull, HSA_WAIT_STATE_ACTIVE) != 0) {
        fprintf(stderr, "completion signal timeout\n");
        return 1;
    }
    spin(seq);
    printf("hsa dispatch ok\n");

    std::vector<double> hip_enq, hip_total, hsa_enq, hsa_total, hsa_sig_total, hip_sync_total;
    for (int round = 0; round < 3; ++round) {
        for (int i = 0; i < n; ++i) {
            const uint32_t s = ++seq;
            double t0 = now_us();
            FlagArgs aa{flag_dev, s, 0};
            hipLaunchKernelGGL(zfec_probe_flag, dim3(1), dim3(64), 0, 0, aa);
            double t1 = now_us();
            spin(s);
            double t2 = now_us();
            hip_enq.push_back(t1 - t0);
            hip_total.push_back(t2 - t0);
        }
        CK(hipDeviceSynchronize());
        for (int i = 0; i < n; ++i) {
            const uint32_t s = ++seq;
            double t0 = now_us();
            FlagArgs aa{flag_dev, s, 0};
            hipLaunchKernelGGL(zfec_probe_flag, dim3(1), dim3(64), 0, 0, aa);
            CK(hipStreamSynchronize(0));
            hip_sync_total.push_back(now_us() - t0);
        }
        for (int i = 0; i < n; ++i) {
            const uint32_t s = ++seq;
            double t0 = now_us();
            dispatch(s, false);
            double t1 = now_us();
            spin(s);
            double t2 = now_us();
            hsa_enq.push_back(t1 - t0);
            hsa_total.push_back(t2 - t0);
        }
        // the queue's last packets are done (flags seen); the signal path
        for (int i = 0; i < n; ++i) {
            const uint32_t s = ++seq;
            double t0 = now_us();
            dispatch(s, true);
            if (hsa_signal_wait_scacquire(done, HSA_SIGNAL_CONDITION_LT, 1, 1000000000ull, HSA_WAIT_STATE_ACTIVE) !=
                0) {
                fprintf(stderr, "completion signal timeout\n");
                return 1;
            }
            hsa_sig_total.push_back(now_us() - t0);
        }
        printf("round %d: hip enqueue %.2f, hip launch->flag %.2f, hip launch+streamsync %.2f, hsa enqueue %.2f, "
               "hsa dispatch->flag %.2f, hsa dispatch->completion signal %.2f us (medians)\n",
               round, median(hip_enq), median(hip_total), median(hip_sync_total), median(hsa_enq), median(hsa_total),
               median(hsa_sig_total));
        hip_enq.clear();
        hip_total.clear();
        hip_sync_total.clear();
        hsa_enq.clear();
        hsa_total.clear();
        hsa_sig_total.clear();
    }
    // drain: every packet signalled its flag, and the last one its signal
    HK(hsa_signal_destroy(done));
    HK(hsa_queue_destroy(q));
    HK(hsa_amd_memory_pool_free(karg));
    HK(hsa_shut_down());
    printf("done\n");
    return 0;
}

// numa_place.hpp -- NUMA placement of the host side of a device's work.
//
// The host-frame paths (fpnn_aes_package_host / _stream_host / the batched classes' flushes)
// gather frames into pinned staging, DMA it, and scatter the results: every byte crosses
// the host memory bus twice and PCIe once.  On a two-socket host a staging arena on the far
// socket, or copy threads running there, sends all of it over the socket interconnect.  The
// engine therefore looks up the NUMA node of its GPU's PCIe function
// (hipDeviceGetPCIBusId -> <sysfs>/bus/pci/devices/<bdf>/numa_node), allocates its pinned
// arenas there (a preferred-node memory policy around hipHostMalloc(hipHostMallocNumaUser))
// and keeps its copy threads on that node's CPUs -- those of them the process may run on.
//
// Host C++ only (no HIP): the CPU tests compile it against a fake sysfs tree
// (tests/cpp/numa_place_test.cpp).
//
//   FPNN_AES_NUMA    auto (default): the GPU's node; off: no placement; <n>: node n
//   FPNN_AES_SYSFS   sysfs root (default /sys; the tests point it at a fake tree)
#pragma once

#include <sched.h>

#include <string>

namespace fpnn_aes {

struct NumaPlacement {
    int node = -1;         // the node the engine's arenas and threads are placed on; -1: none
    int device_node = -1;  // the GPU's node as sysfs reports it (-1: unknown / single node)
    cpu_set_t cpus;        // the node's CPUs this process may run on (copy threads' affinity)
    int ncpus = 0;         // CPU_COUNT(&cpus); 0: threads are not pinned
    std::string why;       // one line: how the placement was chosen
};

// sysfs root (FPNN_AES_SYSFS or "/sys")
std::string sysfs_root();

// NUMA node of a PCI function ("0000:c1:00.0", any case); -1 if unknown
int pci_numa_node(const char *bdf);

// the CPUs of `node` (<sysfs>/devices/system/node/node<n>/cpulist) that the calling
// thread's affinity allows; false if none
bool node_cpus(int node, cpu_set_t *out);

// the placement for a device at `bdf` under FPNN_AES_NUMA (bdf may be null: unknown)
NumaPlacement numa_placement(const char *bdf);

// pin the calling thread to the placement's CPUs (no-op without them); 0 on success
int numa_pin_thread(const NumaPlacement &p);

// While alive, the calling thread's memory policy prefers `node` (MPOL_PREFERRED); the
// previous policy is restored on destruction.  node < 0: no change.
class NumaPreferScope {
public:
    explicit NumaPreferScope(int node);
    ~NumaPreferScope();
    NumaPreferScope(const NumaPreferScope &) = delete;
    NumaPreferScope &operator=(const NumaPreferScope &) = delete;
    bool active() const { return set_; }

private:
    bool set_ = false;
    int old_mode_ = 0;
    unsigned long old_mask_[16] = {};
};

// node holding the page at `p` (after it has been touched); -1 if unknown
int numa_node_of_page(const void *p);

}  // namespace fpnn_aes

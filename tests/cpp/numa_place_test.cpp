// numa_place_test.cpp -- drives fpnn_amd/csrc/numa_place.cpp against a sysfs tree the
// test made (FPNN_AES_SYSFS), without a GPU (tests/test_numa.py).  Prints one JSON object.
//
//   numa_place_test <bdf> [<bdf> ...]
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <string>

#include "../../fpnn_amd/csrc/numa_place.hpp"

using namespace fpnn_aes;

static std::string cpus_json(const cpu_set_t &s) {
    std::string o = "[";
    for (int c = 0; c < CPU_SETSIZE; c++)
        if (CPU_ISSET(c, &s)) o += (o.size() > 1 ? "," : "") + std::to_string(c);
    return o + "]";
}

int main(int argc, char **argv) {
    printf("{\"nodes\": {");
    for (int i = 1; i < argc; i++) printf("%s\"%s\": %d", i > 1 ? ", " : "", argv[i], pci_numa_node(argv[i]));
    printf("}");
    const NumaPlacement p = numa_placement(argc > 1 ? argv[1] : nullptr);
    printf(", \"placement\": {\"node\": %d, \"device_node\": %d, \"ncpus\": %d, \"cpus\": %s, \"why\": \"%s\"}", p.node,
           p.device_node, p.ncpus, cpus_json(p.cpus).c_str(), p.why.c_str());
    // a thread pinned by the placement runs on exactly its CPUs
    cpu_set_t before, after;
    sched_getaffinity(0, sizeof before, &before);
    const int pin = numa_pin_thread(p);
    sched_getaffinity(0, sizeof after, &after);
    printf(", \"pin_rc\": %d, \"affinity_after\": %s", pin, cpus_json(after).c_str());
    sched_setaffinity(0, sizeof before, &before);
    // memory placed under the scope lands on the node; the old policy comes back after it
    const int node = getenv("NUMA_TEST_REAL_NODE") ? atoi(getenv("NUMA_TEST_REAL_NODE")) : 0;
    int page_node = -2, mode_in = -2, mode_after = -2;
    bool active = false;
    {
        NumaPreferScope scope(node);
        active = scope.active();
        unsigned long mask[16];
        syscall(SYS_get_mempolicy, &mode_in, mask, 16 * 8 * sizeof(unsigned long), nullptr, 0UL);
        const size_t n = 1 << 20;
        char *buf = static_cast<char *>(aligned_alloc(4096, n));
        memset(buf, 1, n);
        page_node = numa_node_of_page(buf + n / 2);
        free(buf);
    }
    unsigned long mask[16];
    syscall(SYS_get_mempolicy, &mode_after, mask, 16 * 8 * sizeof(unsigned long), nullptr, 0UL);
    printf(", \"prefer\": {\"node\": %d, \"active\": %s, \"mode_in\": %d, \"mode_after\": %d, \"page_node\": %d}}\n", node,
           active ? "true" : "false", mode_in, mode_after, page_node);
    return 0;
}

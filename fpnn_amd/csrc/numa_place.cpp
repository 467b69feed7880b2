// numa_place.cpp -- see numa_place.hpp.  Plain syscalls (no libnuma in the image).
#include "numa_place.hpp"

#include <ctype.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>

namespace fpnn_aes {

namespace {

constexpr int kMpolDefault = 0, kMpolPreferred = 1;
constexpr unsigned long kMaskBits = 16 * 8 * sizeof(unsigned long);

bool read_line(const std::string &path, std::string *out) {
    FILE *f = fopen(path.c_str(), "r");
    if (!f) return false;
    char buf[4096];
    const bool ok = fgets(buf, sizeof buf, f) != nullptr;
    fclose(f);
    if (!ok) return false;
    out->assign(buf);
    while (!out->empty() && isspace((unsigned char)out->back())) out->pop_back();
    return true;
}

// "0-15,32-47" -> set bits; false on a malformed list
bool parse_cpulist(const std::string &s, cpu_set_t *out) {
    CPU_ZERO(out);
    const char *p = s.c_str();
    while (*p) {
        char *end = nullptr;
        const long a = strtol(p, &end, 10);
        if (end == p || a < 0) return false;
        long b = a;
        p = end;
        if (*p == '-') {
            b = strtol(p + 1, &end, 10);
            if (end == p + 1 || b < a) return false;
            p = end;
        }
        for (long c = a; c <= b && c < CPU_SETSIZE; c++) CPU_SET((int)c, out);
        if (*p == ',') p++;
        else if (*p) return false;
    }
    return true;
}

}  // namespace

std::string sysfs_root() {
    const char *v = getenv("FPNN_AES_SYSFS");
    return (v && *v) ? std::string(v) : std::string("/sys");
}

int pci_numa_node(const char *bdf) {
    if (!bdf || !*bdf) return -1;
    std::string id(bdf);
    for (auto &c : id) c = (char)tolower((unsigned char)c);
    std::string line;
    if (!read_line(sysfs_root() + "/bus/pci/devices/" + id + "/numa_node", &line)) return -1;
    char *end = nullptr;
    const long n = strtol(line.c_str(), &end, 10);
    if (end == line.c_str() || n < 0 || n >= (long)kMaskBits) return -1;  // "-1": no affinity
    return (int)n;
}

bool node_cpus(int node, cpu_set_t *out) {
    CPU_ZERO(out);
    if (node < 0) return false;
    std::string line;
    if (!read_line(sysfs_root() + "/devices/system/node/node" + std::to_string(node) + "/cpulist", &line))
        return false;
    cpu_set_t mine, on_node;
    if (!parse_cpulist(line, &on_node)) return false;
    if (sched_getaffinity(0, sizeof mine, &mine) != 0) return false;
    CPU_AND(out, &on_node, &mine);
    return CPU_COUNT(out) > 0;
}

NumaPlacement numa_placement(const char *bdf) {
    NumaPlacement p;
    CPU_ZERO(&p.cpus);
    p.device_node = pci_numa_node(bdf);
    const char *v = getenv("FPNN_AES_NUMA");
    const std::string mode = v ? v : "auto";
    if (mode == "off") {
        p.why = "FPNN_AES_NUMA=off";
        return p;
    }
    if (mode != "auto") {
        char *end = nullptr;
        const long n = strtol(mode.c_str(), &end, 10);
        if (end == mode.c_str() || *end || n < 0 || n >= (long)kMaskBits) {
            p.why = "FPNN_AES_NUMA=" + mode + " not understood: no placement";
            return p;
        }
        p.node = (int)n;
        p.why = "FPNN_AES_NUMA=" + mode;
    } else if (p.device_node >= 0) {
        p.node = p.device_node;
        p.why = std::string("device ") + (bdf ? bdf : "?") + " on node " + std::to_string(p.node);
    } else {
        p.why = std::string("no NUMA node for device ") + (bdf ? bdf : "?") + ": no placement";
        return p;
    }
    if (node_cpus(p.node, &p.cpus)) {
        p.ncpus = CPU_COUNT(&p.cpus);
    } else {
        p.why += "; none of the node's CPUs in this process's affinity: copy threads unpinned";
    }
    return p;
}

int numa_pin_thread(const NumaPlacement &p) {
    if (p.ncpus <= 0) return 0;
    return pthread_setaffinity_np(pthread_self(), sizeof p.cpus, &p.cpus);
}

NumaPreferScope::NumaPreferScope(int node) {
    if (node < 0 || (unsigned long)node >= kMaskBits) return;
    if (syscall(SYS_get_mempolicy, &old_mode_, old_mask_, kMaskBits, nullptr, 0UL) != 0) return;
    unsigned long mask[16] = {};
    mask[node / (8 * sizeof(unsigned long))] = 1UL << (node % (8 * sizeof(unsigned long)));
    // (maxnode counts one past the last bit the kernel reads)
    set_ = syscall(SYS_set_mempolicy, kMpolPreferred, mask, kMaskBits + 1) == 0;
}

NumaPreferScope::~NumaPreferScope() {
    if (!set_) return;
    if (old_mode_ == kMpolDefault)
        (void)syscall(SYS_set_mempolicy, kMpolDefault, nullptr, 0UL);
    else
        (void)syscall(SYS_set_mempolicy, old_mode_, old_mask_, kMaskBits + 1);
}

int numa_node_of_page(const void *p) {
    void *pages[1] = {const_cast<void *>(p)};
    int status[1] = {-1};
    if (syscall(SYS_move_pages, 0, 1UL, pages, nullptr, status, 0) != 0) return -1;
    return status[0] >= 0 ? status[0] : -1;
}

}  // namespace fpnn_aes

// Per-GPU host data plane: which CPUs each GPU worker's host threads (ingest sockets, bitstream
// parse strands, intra-picture fan-out, GPU feeder / lanes, frame-bus pump) run on, and how many
// parse threads it gets.
//
// The reference scales CPU with cameras (one Docker container per camera, each with its own CPU
// share: server/services/rtsp_process_manager.go:70-81,106-115). Here the unit is the GPU: every
// Worker owns a host domain sized cpu_budget / n_workers (no constant cap) and pinned to the
// GPU's NUMA-local CPUs (PCI BDF from hipDeviceGetPCIBusId -> /sys/bus/pci/devices/<bdf>/
// local_cpulist), so parse threads, the pinned access-unit / record pools they fill (hipHostMalloc
// places them on the node of the thread's current device) and the GPU that pulls the records over
// PCIe sit on one socket, and decode capacity grows with the number of GPUs instead of stopping at
// one process-wide pool.
#pragma once

#include <functional>
#include <string>
#include <vector>

#include "common.h"

namespace vep {

struct HostDomain {
  int device = -1;            // GPU ordinal (-1: CPU backend)
  int index = 0;              // worker index in the plan
  int numa_node = -1;         // the GPU's NUMA node (-1: unknown)
  std::string pci_bus_id;     // "0000:05:00.0" ("" unknown)
  std::vector<int> cpus;      // CPUs the domain's host threads run on (empty: not pinned)
  int cpu_share = 0;          // CPUs of the process's budget (affinity and cgroup quota) it gets
  int parse_threads = 0;      // parse strand pool (0: the process-wide default pool)
  int io_threads = 0;         // epoll socket loops
  std::string source;         // numa | split | explicit
};

// CPUs in this process's affinity mask, ascending.
std::vector<int> affinity_cpus();
// "0-3,8,10-11" <-> {0,1,2,3,8,10,11}
std::vector<int> parse_cpulist(const std::string& s);
std::string format_cpulist(const std::vector<int>& cpus);
// The GPU's PCI bus id and sysfs-reported local CPUs / NUMA node ({} / -1 when unknown).
std::string gpu_pci_bus_id(int device);
std::vector<int> gpu_local_cpus(int device, int* numa_node = nullptr);

// One domain per entry of `devices` (a device may repeat: several workers per GPU). CPU sets:
//  * explicit[i] when given (config gpu.host_cpus / VEP_HOST_CPUS "0-7;8-15;..."), intersected
//    with the affinity mask;
//  * else the GPU's local CPUs intersected with the affinity mask, split into contiguous equal
//    parts among the workers that share that local set;
//  * else (CPU backend, no sysfs) the affinity CPUs not claimed above, split evenly.
// cpu_share is the set's size, or its proportional part of a cgroup quota smaller than the CPUs the
// sets cover (a 16-CPU quota on a 256-CPU mask: one domain gets 16, eight get 2 each); parse threads =
// cpu_share - reserve (at least 1; reserve only when the share is 4..15: from 16 CPUs the ingest /
// worker / lane threads take ~0.2 cores of the timed region, and a parse thread on every CPU of
// the share measured +3-4% decoded pictures/s, profiles/r6/threads/), io threads 1 (2 from 16).
// VEP_INGEST_PARSE_THREADS / VEP_IO_THREADS override the sizes.
std::vector<HostDomain> plan_host_domains(const std::vector<int>& devices,
                                          const std::vector<std::string>& explicit_cpus = {}, int reserve = 1);

// Pin the calling thread to `cpus` (no-op for an empty list or one the mask does not allow).
void pin_current_thread(const std::vector<int>& cpus);

// Called first on every thread a domain's pools start: pins it, makes the domain's GPU current
// (pinned host allocations land on its NUMA node) and binds the domain's fan-out pool.
std::function<void()> domain_thread_init(const HostDomain& d, class FanOut* fan);

}  // namespace vep

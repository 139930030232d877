// Per-GPU host domains. See hostplan.h.
#include "hostplan.h"

#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <fstream>
#include <map>
#include <set>
#include <sstream>

#include "fanout.h"
#include "hostmem.h"
#include "ioloop.h"

namespace vep {

std::vector<int> affinity_cpus() {
  std::vector<int> out;
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof set, &set) == 0)
    for (int c = 0; c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, &set)) out.push_back(c);
  return out;
}

std::vector<int> parse_cpulist(const std::string& s) {
  std::set<int> out;
  std::stringstream ss(s);
  std::string part;
  while (std::getline(ss, part, ',')) {
    part.erase(std::remove_if(part.begin(), part.end(), [](unsigned char ch) { return std::isspace(ch); }), part.end());
    if (part.empty()) continue;
    const size_t dash = part.find('-');
    char* end = nullptr;
    const long a = std::strtol(part.c_str(), &end, 10);
    VEP_CHECK(end != part.c_str() && a >= 0 && a < CPU_SETSIZE, "bad CPU list '" + s + "'");
    long b = a;
    if (dash != std::string::npos) {
      b = std::strtol(part.c_str() + dash + 1, &end, 10);
      VEP_CHECK(b >= a && b < CPU_SETSIZE, "bad CPU list '" + s + "'");
    }
    for (long c = a; c <= b; ++c) out.insert(int(c));
  }
  return {out.begin(), out.end()};
}

std::string format_cpulist(const std::vector<int>& cpus) {
  std::string out;
  for (size_t i = 0; i < cpus.size();) {
    size_t j = i;
    while (j + 1 < cpus.size() && cpus[j + 1] == cpus[j] + 1) ++j;
    if (!out.empty()) out += ',';
    out += std::to_string(cpus[i]);
    if (j > i) out += '-' + std::to_string(cpus[j]);
    i = j + 1;
  }
  return out;
}

std::string gpu_pci_bus_id(int device) {
  if (device < 0) return "";
  char buf[64] = {0};
  if (hipDeviceGetPCIBusId(buf, int(sizeof buf), device) != hipSuccess) {
    (void)hipGetLastError();
    return "";
  }
  std::string id(buf);
  for (char& c : id) c = char(std::tolower(static_cast<unsigned char>(c)));
  return id;
}

std::vector<int> gpu_local_cpus(int device, int* numa_node) {
  if (numa_node) *numa_node = -1;
  const std::string bdf = gpu_pci_bus_id(device);
  if (bdf.empty()) return {};
  const std::string dir = "/sys/bus/pci/devices/" + bdf;
  std::ifstream f(dir + "/local_cpulist");
  std::string line;
  if (!f || !std::getline(f, line)) return {};
  if (numa_node) {
    std::ifstream n(dir + "/numa_node");
    int node = -1;
    if (n >> node) *numa_node = node;
  }
  try {
    return parse_cpulist(line);
  } catch (const std::exception&) {
    return {};
  }
}

static std::vector<int> intersect(const std::vector<int>& a, const std::vector<int>& b) {
  std::vector<int> out;
  std::set_intersection(a.begin(), a.end(), b.begin(), b.end(), std::back_inserter(out));
  return out;
}

// k contiguous, near-equal parts of `cpus` (part j of k)
static std::vector<int> part_of(const std::vector<int>& cpus, int j, int k) {
  const size_t n = cpus.size();
  const size_t a = n * size_t(j) / size_t(k), b = n * size_t(j + 1) / size_t(k);
  return {cpus.begin() + long(a), cpus.begin() + long(b)};
}

static int env_int(const char* name) {
  const char* v = std::getenv(name);
  return v && *v ? std::max(1, std::atoi(v)) : 0;
}

std::vector<HostDomain> plan_host_domains(const std::vector<int>& devices, const std::vector<std::string>& explicit_cpus,
                                          int reserve) {
  const std::vector<int> aff = affinity_cpus();
  const int n = int(devices.size());
  std::vector<HostDomain> out(static_cast<size_t>(n));
  std::vector<std::vector<int>> local(static_cast<size_t>(n));
  for (int i = 0; i < n; ++i) {
    HostDomain& d = out[size_t(i)];
    d.device = devices[size_t(i)];
    d.index = i;
    if (size_t(i) < explicit_cpus.size() && !explicit_cpus[size_t(i)].empty()) {
      d.cpus = intersect(parse_cpulist(explicit_cpus[size_t(i)]), aff);
      d.source = "explicit";
    }
    if (d.device >= 0) {
      d.pci_bus_id = gpu_pci_bus_id(d.device);
      local[size_t(i)] = intersect(gpu_local_cpus(d.device, &d.numa_node), aff);
    }
  }
  // workers of GPUs with the same local CPU set split it
  std::map<std::vector<int>, std::vector<int>> groups;
  for (int i = 0; i < n; ++i)
    if (out[size_t(i)].source.empty() && !local[size_t(i)].empty()) groups[local[size_t(i)]].push_back(i);
  for (const auto& [cpus, members] : groups) {
    const int k = int(members.size());
    if (int(cpus.size()) < k) continue;  // (fewer CPUs than workers: left to the even split)
    for (int j = 0; j < k; ++j) {
      HostDomain& d = out[size_t(members[size_t(j)])];
      d.cpus = part_of(cpus, j, k);
      d.source = "numa";
    }
  }
  // the rest split what nobody claimed (or everything, when that is too little)
  std::vector<int> rest_idx;
  std::set<int> claimed;
  for (const HostDomain& d : out) {
    if (d.source.empty()) rest_idx.push_back(d.index);
    else claimed.insert(d.cpus.begin(), d.cpus.end());
  }
  if (!rest_idx.empty()) {
    std::vector<int> pool;
    for (int c : aff)
      if (!claimed.count(c)) pool.push_back(c);
    if (pool.size() < rest_idx.size()) pool = aff;
    const int k = int(rest_idx.size());
    for (int j = 0; j < k; ++j) {
      HostDomain& d = out[size_t(rest_idx[size_t(j)])];
      d.cpus = int(pool.size()) >= k ? part_of(pool, j, k) : pool;
      d.source = "split";
    }
  }
  // sizes: each domain's part of the process budget (a cgroup quota below the CPUs the domains
  // cover is shared in proportion to their sets)
  const int budget = cpu_budget();
  std::set<int> covered;
  for (const HostDomain& d : out) covered.insert(d.cpus.begin(), d.cpus.end());
  const i64 cover = i64(covered.size());
  const int parse_env = env_int("VEP_INGEST_PARSE_THREADS"), io_env = env_int("VEP_IO_THREADS");
  for (HostDomain& d : out) {
    int share = int(d.cpus.size());
    if (cover > 0 && budget < cover) {
      i64 sum = 0;  // (sets may overlap when CPUs are scarce: divide by the sum of the sets)
      for (const HostDomain& e : out) sum += i64(e.cpus.size());
      share = int((i64(d.cpus.size()) * budget + sum / 2) / std::max<i64>(1, sum));
    }
    d.cpu_share = std::max(1, share);
    d.parse_threads = parse_env ? parse_env
                                : std::max(1, d.cpu_share - (d.cpu_share >= 4 && d.cpu_share < 16 ? reserve : 0));
    d.io_threads = io_env ? io_env : (d.cpu_share >= 16 ? 2 : 1);
  }
  return out;
}

void pin_current_thread(const std::vector<int>& cpus) {
  if (cpus.empty()) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus)
    if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &set);
  (void)sched_setaffinity(0, sizeof set, &set);  // (0: the calling thread)
}

std::function<void()> domain_thread_init(const HostDomain& d, FanOut* fan) {
  const std::vector<int> cpus = d.cpus;
  const int dev = d.device;
  return [cpus, dev, fan] {
    pin_current_thread(cpus);
    if (dev >= 0 && hipSetDevice(dev) != hipSuccess) (void)hipGetLastError();
    hostmem::bind_thread_device(dev);
    FanOut::bind_thread(fan);
  };
}

}  // namespace vep

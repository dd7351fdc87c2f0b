// mi355x_launch: native multi-process launcher, one process per GPU.
//
// Replaces the reference's `mpirun -np 8 ... smddprun python -m mpi4py <entry>` (captured at
// notebooks/2_pytorch_dist_smddp_gpu.ipynb log):
//   * forks --nproc ranks, each with RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE /
//     MASTER_ADDR / MASTER_PORT (torch.distributed env:// rendezvous) and
//     OMPI_COMM_WORLD_{RANK,SIZE,LOCAL_RANK} for MPI-style scripts;
//   * optional per-rank CPU affinity (--bind-cpus), GPU/NUMA-aware: local rank r drives GPU r, so
//     it is bound to CPUs of that GPU's NUMA node (sysfs: the AMD GPUs under /sys/class/drm in
//     PCI order -> device/numa_node; /sys/devices/system/node/nodeN/cpulist), the node's allowed
//     CPUs split evenly among the ranks whose GPUs sit on it; contiguous equal slices of the
//     allowed set when the topology is unreadable (the reference pinned each rank to its GPU's
//     socket: CPU affinity ff,ffff0000,00ffffff, nb2:380).  --print-binding prints the plan.
//   * `--tag-output` prefixes every line as "[1,mpirank:R,HOST]<stdout>:" / "<stderr>:";
//   * abort-on-non-zero-status: the first rank that exits non-zero (or dies by a signal)
//     makes the launcher SIGTERM (then SIGKILL after --grace seconds) every other rank,
//     and the launcher exits with that rank's code (orte_abort_on_non_zero_status 1);
//   * SIGINT/SIGTERM to the launcher are forwarded to all ranks.
// The launcher itself never touches the GPU; children exec the command before any GPU init.
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <sched.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <dirent.h>
#include <fstream>
#include <map>
#include <set>
#include <sstream>
#include <string>
#include <vector>

namespace {

struct Rank {
  pid_t pid = -1;
  int out_fd = -1, err_fd = -1;
  std::string out_buf, err_buf;
  bool done = false;
  int status = 0;
};

volatile sig_atomic_t g_signal = 0;
void on_signal(int s) { g_signal = s; }

void usage() {
  fprintf(stderr,
          "usage: mi355x_launch --nproc N [--node-rank R --nnodes M] [--master-addr A] [--master-port P]\n"
          "                     [--host NAME] [--tag-output] [--bind-cpus] [--print-binding] [--grace SEC]\n"
          "                     [-x KEY=VAL]...\n"
          "                     [--rank-env KEY=PREFIX]... -- cmd args...\n");
}

void emit(Rank& r, int rank, const char* host, bool is_err, bool tag, bool flush_all) {
  std::string& buf = is_err ? r.err_buf : r.out_buf;
  FILE* f = is_err ? stderr : stdout;
  size_t pos;
  while ((pos = buf.find('\n')) != std::string::npos || (flush_all && !buf.empty())) {
    std::string line = pos == std::string::npos ? buf : buf.substr(0, pos);
    buf.erase(0, pos == std::string::npos ? buf.size() : pos + 1);
    if (tag)
      fprintf(f, "[1,mpirank:%d,%s]<%s>:%s\n", rank, host, is_err ? "stderr" : "stdout", line.c_str());
    else
      fprintf(f, "%s\n", line.c_str());
  }
  fflush(f);
}

std::vector<int> allowed_cpus() {
  std::vector<int> cpus;
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) == 0)
    for (int c = 0; c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, &set)) cpus.push_back(c);
  return cpus;
}

// ------------------------------------------------------------ GPU / NUMA topology
// MI355X_DP_TOPO_ROOT prefixes every sysfs path (tests build a fake tree).
std::string topo_root() {
  const char* r = getenv("MI355X_DP_TOPO_ROOT");
  return r ? std::string(r) : std::string();
}

bool read_file(const std::string& path, std::string& out) {
  std::ifstream f(path);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  out = ss.str();
  while (!out.empty() && (out.back() == '\n' || out.back() == ' ')) out.pop_back();
  return true;
}

std::vector<int> parse_cpulist(const std::string& s) {  // "0-3,8,10-11"
  std::vector<int> v;
  std::stringstream ss(s);
  std::string part;
  while (std::getline(ss, part, ',')) {
    if (part.empty()) continue;
    size_t d = part.find('-');
    int a = atoi(part.c_str()), b = d == std::string::npos ? a : atoi(part.c_str() + d + 1);
    for (int c = a; c <= b; ++c) v.push_back(c);
  }
  return v;
}

// NUMA node of every AMD GPU (vendor 0x1002, display 0x03xxxx or accelerator 0x12xxxx class), in
// PCI-address order = HIP device order; empty if sysfs is unreadable
std::vector<int> gpu_numa_nodes() {
  const std::string base = topo_root() + "/sys/class/drm";
  std::vector<std::pair<std::string, int>> gpus;
  std::set<std::string> seen;
  DIR* d = opendir(base.c_str());
  if (!d) return {};
  while (dirent* e = readdir(d)) {
    std::string n = e->d_name;
    if (n.rfind("card", 0) != 0 || n.find('-') != std::string::npos) continue;
    const std::string dev = base + "/" + n + "/device";
    std::string vendor, cls, numa, link;
    if (!read_file(dev + "/vendor", vendor) || vendor != "0x1002") continue;
    if (!read_file(dev + "/class", cls) || !(cls.rfind("0x03", 0) == 0 || cls.rfind("0x12", 0) == 0)) continue;
    char buf[4096];
    ssize_t k = readlink(dev.c_str(), buf, sizeof(buf) - 1);
    link = k > 0 ? std::string(buf, k) : n;
    link = link.substr(link.find_last_of('/') + 1);  // PCI address, e.g. 0000:05:00.0
    if (!seen.insert(link).second) continue;
    int node = read_file(dev + "/numa_node", numa) ? atoi(numa.c_str()) : 0;
    gpus.emplace_back(link, node < 0 ? 0 : node);
  }
  closedir(d);
  std::sort(gpus.begin(), gpus.end());
  std::vector<int> out;
  for (auto& g : gpus) out.push_back(g.second);
  return out;
}

std::vector<int> node_cpus(int node) {
  std::string s;
  if (!read_file(topo_root() + "/sys/devices/system/node/node" + std::to_string(node) + "/cpulist", s)) return {};
  return parse_cpulist(s);
}

// CPU set of every local rank: GPU/NUMA-aware when the topology is readable, else equal slices
std::vector<std::vector<int>> plan_binding(int nproc, const std::vector<int>& allowed, std::string& how) {
  std::vector<std::vector<int>> plan(nproc);
  const std::vector<int> numa = gpu_numa_nodes();
  std::set<int> allow(allowed.begin(), allowed.end());
  bool ok = !numa.empty();
  if (ok) {
    std::map<int, std::vector<int>> ranks_on;  // node -> local ranks whose GPU is on it
    for (int r = 0; r < nproc; ++r) ranks_on[numa[r % numa.size()]].push_back(r);
    for (auto& kv : ranks_on) {
      std::vector<int> cpus;
      for (int c : node_cpus(kv.first))
        if (allow.count(c)) cpus.push_back(c);
      if (cpus.empty()) { ok = false; break; }
      const int k = (int)kv.second.size();
      const int per = std::max<int>(1, (int)cpus.size() / k);
      for (int j = 0; j < k; ++j)
        for (int c = j * per; c < (j + 1) * per && c < (int)cpus.size(); ++c) plan[kv.second[j]].push_back(cpus[c]);
    }
  }
  if (ok) {
    how = "numa";
    return plan;
  }
  how = "slices";
  plan.assign(nproc, {});
  const int per = std::max<int>(1, (int)allowed.size() / nproc);
  for (int r = 0; r < nproc; ++r)
    for (int c = r * per; c < (r + 1) * per && c < (int)allowed.size(); ++c) plan[r].push_back(allowed[c]);
  return plan;
}

}  // namespace

int main(int argc, char** argv) {
  int nproc = 1, node_rank = 0, nnodes = 1, grace = 10;
  std::string master_addr = "127.0.0.1", master_port = "29500", host = "algo-1";
  bool tag = false, bind = false, print_binding = false;
  std::vector<std::string> extra_env, rank_env;
  int i = 1;
  for (; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&](void) -> std::string {
      if (i + 1 >= argc) { usage(); exit(2); }
      return argv[++i];
    };
    if (a == "--") { ++i; break; }
    else if (a == "--nproc" || a == "-np") nproc = atoi(next().c_str());
    else if (a == "--node-rank") node_rank = atoi(next().c_str());
    else if (a == "--nnodes") nnodes = atoi(next().c_str());
    else if (a == "--master-addr") master_addr = next();
    else if (a == "--master-port") master_port = next();
    else if (a == "--host") host = next();
    else if (a == "--grace") grace = atoi(next().c_str());
    else if (a == "--tag-output") tag = true;
    else if (a == "--bind-cpus") bind = true;
    else if (a == "--print-binding") print_binding = true;
    else if (a == "-x") extra_env.push_back(next());
    else if (a == "--rank-env") rank_env.push_back(next());  // KEY=PREFIX -> KEY=PREFIX<rank+1>
    else { fprintf(stderr, "unknown option %s\n", a.c_str()); usage(); return 2; }
  }
  std::vector<int> cpus = allowed_cpus();
  std::string how;
  const std::vector<std::vector<int>> binding = plan_binding(std::max(1, nproc), cpus, how);
  if (print_binding) {
    for (int r = 0; r < nproc; ++r) {
      printf("rank %d (%s):", r, how.c_str());
      for (int c : binding[r]) printf(" %d", c);
      printf("\n");
    }
    return 0;
  }
  if (i >= argc || nproc < 1) { usage(); return 2; }
  char** cmd = argv + i;
  const int world = nproc * nnodes;

  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_handler = on_signal;
  sigaction(SIGINT, &sa, nullptr);
  sigaction(SIGTERM, &sa, nullptr);
  signal(SIGPIPE, SIG_IGN);

  std::vector<Rank> ranks(nproc);
  for (int lr = 0; lr < nproc; ++lr) {
    int po[2], pe[2];
    if (pipe(po) || pipe(pe)) { perror("pipe"); return 1; }
    pid_t pid = fork();
    if (pid < 0) { perror("fork"); return 1; }
    if (pid == 0) {
      setpgid(0, 0);
      dup2(po[1], 1);
      dup2(pe[1], 2);
      close(po[0]); close(po[1]); close(pe[0]); close(pe[1]);
      const int rank = node_rank * nproc + lr;
      auto set = [](const char* k, const std::string& v) { setenv(k, v.c_str(), 1); };
      set("RANK", std::to_string(rank));
      set("LOCAL_RANK", std::to_string(lr));
      set("WORLD_SIZE", std::to_string(world));
      set("LOCAL_WORLD_SIZE", std::to_string(nproc));
      set("GROUP_RANK", std::to_string(node_rank));
      set("MASTER_ADDR", master_addr);
      set("MASTER_PORT", master_port);
      set("OMPI_COMM_WORLD_RANK", std::to_string(rank));
      set("OMPI_COMM_WORLD_SIZE", std::to_string(world));
      set("OMPI_COMM_WORLD_LOCAL_RANK", std::to_string(lr));
      set("OMPI_COMM_WORLD_LOCAL_SIZE", std::to_string(nproc));
      for (auto& kv : extra_env) {
        size_t eq = kv.find('=');
        if (eq != std::string::npos) setenv(kv.substr(0, eq).c_str(), kv.substr(eq + 1).c_str(), 1);
      }
      for (auto& kv : rank_env) {
        size_t eq = kv.find('=');
        if (eq != std::string::npos)
          setenv(kv.substr(0, eq).c_str(), (kv.substr(eq + 1) + std::to_string(rank + 1)).c_str(), 1);
      }
      if (bind && !binding[lr].empty()) {
        cpu_set_t set_;
        CPU_ZERO(&set_);
        for (int c : binding[lr]) CPU_SET(c, &set_);
        sched_setaffinity(0, sizeof(set_), &set_);
        set("OMP_NUM_THREADS", std::to_string(binding[lr].size()));
      }
      execvp(cmd[0], cmd);
      fprintf(stderr, "mi355x_launch: exec %s failed: %s\n", cmd[0], strerror(errno));
      _exit(127);
    }
    close(po[1]);
    close(pe[1]);
    ranks[lr].pid = pid;
    ranks[lr].out_fd = po[0];
    ranks[lr].err_fd = pe[0];
  }

  int exit_code = 0, failed_rank = -1, alive = nproc;
  time_t kill_deadline = 0;
  bool terminating = false;
  auto terminate_all = [&](int sig) {
    for (auto& r : ranks)
      if (!r.done && r.pid > 0) kill(-r.pid, sig);
  };

  char buf[65536];
  while (alive > 0) {
    std::vector<pollfd> fds;
    std::vector<std::pair<int, bool>> owner;
    for (int lr = 0; lr < nproc; ++lr) {
      if (ranks[lr].out_fd >= 0) { fds.push_back({ranks[lr].out_fd, POLLIN, 0}); owner.push_back({lr, false}); }
      if (ranks[lr].err_fd >= 0) { fds.push_back({ranks[lr].err_fd, POLLIN, 0}); owner.push_back({lr, true}); }
    }
    if (!fds.empty()) poll(fds.data(), fds.size(), 200);
    else usleep(50000);
    for (size_t k = 0; k < fds.size(); ++k) {
      if (!(fds[k].revents & (POLLIN | POLLHUP | POLLERR))) continue;
      Rank& r = ranks[owner[k].first];
      ssize_t n = read(fds[k].fd, buf, sizeof(buf));
      const int rank = node_rank * nproc + owner[k].first;
      if (n > 0) {
        (owner[k].second ? r.err_buf : r.out_buf).append(buf, n);
        emit(r, rank, host.c_str(), owner[k].second, tag, false);
      } else {
        emit(r, rank, host.c_str(), owner[k].second, tag, true);
        close(fds[k].fd);
        (owner[k].second ? r.err_fd : r.out_fd) = -1;
      }
    }
    int st;
    pid_t p;
    while ((p = waitpid(-1, &st, WNOHANG)) > 0) {
      for (int lr = 0; lr < nproc; ++lr) {
        Rank& r = ranks[lr];
        if (r.pid != p || r.done) continue;
        r.done = true;
        r.status = st;
        --alive;
        int code = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + (WIFSIGNALED(st) ? WTERMSIG(st) : 0);
        if (code != 0 && failed_rank < 0) {
          failed_rank = node_rank * nproc + lr;
          exit_code = code;
          fprintf(stderr, "mi355x_launch: rank %d exited with status %d; aborting all ranks\n", failed_rank, code);
          terminating = true;
          terminate_all(SIGTERM);
          kill_deadline = time(nullptr) + grace;
        }
      }
    }
    if (g_signal && !terminating) {
      fprintf(stderr, "mi355x_launch: caught signal %d, forwarding to ranks\n", (int)g_signal);
      terminating = true;
      terminate_all(SIGTERM);
      kill_deadline = time(nullptr) + grace;
      if (exit_code == 0) exit_code = 128 + g_signal;
    }
    if (terminating && kill_deadline && time(nullptr) >= kill_deadline) {
      terminate_all(SIGKILL);
      kill_deadline = 0;
    }
  }
  // drain remaining output
  for (int lr = 0; lr < nproc; ++lr) {
    Rank& r = ranks[lr];
    for (int* fd : {&r.out_fd, &r.err_fd}) {
      if (*fd < 0) continue;
      ssize_t n;
      while ((n = read(*fd, buf, sizeof(buf))) > 0) (fd == &r.err_fd ? r.err_buf : r.out_buf).append(buf, n);
      close(*fd);
      *fd = -1;
    }
    emit(r, node_rank * nproc + lr, host.c_str(), false, tag, true);
    emit(r, node_rank * nproc + lr, host.c_str(), true, tag, true);
  }
  return exit_code;
}

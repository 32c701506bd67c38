// polyflow process supervisor: spawn trial replicas and wait for ANY of them to exit, event-driven.
//
// The reference learns about a trial's end through a Kubernetes pod watch -> AMQP -> Celery worker chain
// (polyaxon/monitor_statuses/monitor.py:57-135, events_handlers/tasks/statuses.py:23-60) plus a 30 s
// reconciliation cron (crons/tasks/experiments.py:9-17).  On one node the kernel already knows the
// instant a child exits: this library spawns each replica with posix_spawn in its own process group
// (stdout+stderr appended to its log file), holds a pidfd for it, and `plx_pm_wait` blocks in epoll on
// all pidfds at once (plus an eventfd so the scheduler can wake it), so the scheduler reacts to an exit in
// microseconds with no polling and no thread per child.
//
// C ABI (ctypes):
//   plx_pm_create() -> handle            plx_pm_destroy(h)
//   plx_pm_spawn(h, argv, envp, cwd, log_path, &pid) -> 0 | errno
//   plx_pm_wait(h, timeout_ms, &pid, &status) -> 1 exited / 0 timeout / 2 woken / <0 error
//   plx_pm_wake(h)                        plx_pm_signal(h, pid, sig, group)
//   plx_pm_count(h) -> live children
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <spawn.h>
#include <stdint.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/syscall.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <unistd.h>

#include <mutex>
#include <unordered_map>

#define PLX_API extern "C" __attribute__((visibility("default")))

#ifndef SYS_pidfd_open
#define SYS_pidfd_open 434
#endif

namespace {

struct Monitor {
  int ep = -1;
  int wake_fd = -1;
  std::mutex mu;
  std::unordered_map<int, pid_t> fd_to_pid;  // pidfd -> pid
  std::unordered_map<pid_t, int> pid_to_fd;
};

int pidfd_open(pid_t pid) { return (int)syscall(SYS_pidfd_open, pid, 0); }

}  // namespace

PLX_API void* plx_pm_create() {
  Monitor* m = new Monitor();
  m->ep = epoll_create1(EPOLL_CLOEXEC);
  m->wake_fd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (m->ep < 0 || m->wake_fd < 0) {
    delete m;
    return nullptr;
  }
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = m->wake_fd;
  epoll_ctl(m->ep, EPOLL_CTL_ADD, m->wake_fd, &ev);
  return m;
}

PLX_API void plx_pm_destroy(void* h) {
  Monitor* m = static_cast<Monitor*>(h);
  if (!m) return;
  for (auto& kv : m->fd_to_pid) close(kv.first);
  close(m->ep);
  close(m->wake_fd);
  delete m;
}

PLX_API int plx_pm_spawn(void* h, char* const* argv, char* const* envp, const char* cwd, const char* log_path,
                         int* out_pid) {
  Monitor* m = static_cast<Monitor*>(h);
  posix_spawn_file_actions_t fa;
  posix_spawnattr_t attr;
  posix_spawn_file_actions_init(&fa);
  posix_spawnattr_init(&attr);
  if (log_path && *log_path) {
    posix_spawn_file_actions_addopen(&fa, 1, log_path, O_WRONLY | O_CREAT | O_APPEND, 0644);
    posix_spawn_file_actions_adddup2(&fa, 1, 2);
  }
  posix_spawn_file_actions_addopen(&fa, 0, "/dev/null", O_RDONLY, 0);
  if (cwd && *cwd) posix_spawn_file_actions_addchdir_np(&fa, cwd);
  // own process group so stop() can signal the whole replica tree (launcher + its children)
  posix_spawnattr_setpgroup(&attr, 0);
  sigset_t def;
  sigemptyset(&def);
  sigaddset(&def, SIGTERM);
  sigaddset(&def, SIGINT);
  sigaddset(&def, SIGCHLD);
  sigaddset(&def, SIGPIPE);
  posix_spawnattr_setsigdefault(&attr, &def);
  sigset_t none;
  sigemptyset(&none);
  posix_spawnattr_setsigmask(&attr, &none);
  posix_spawnattr_setflags(&attr, POSIX_SPAWN_SETPGROUP | POSIX_SPAWN_SETSIGDEF | POSIX_SPAWN_SETSIGMASK);
  pid_t pid = 0;
  int rc = posix_spawnp(&pid, argv[0], &fa, &attr, argv, envp);
  posix_spawn_file_actions_destroy(&fa);
  posix_spawnattr_destroy(&attr);
  if (rc != 0) return rc;
  int pfd = pidfd_open(pid);
  if (pfd < 0) {  // cannot supervise it: do not leak an unreaped child
    const int e = errno ? errno : -1;
    kill(pid, SIGKILL);
    waitpid(pid, nullptr, 0);
    return e;
  }
  {
    std::lock_guard<std::mutex> lk(m->mu);
    m->fd_to_pid[pfd] = pid;
    m->pid_to_fd[pid] = pfd;
  }
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = pfd;
  epoll_ctl(m->ep, EPOLL_CTL_ADD, pfd, &ev);
  *out_pid = (int)pid;
  return 0;
}

// Reap one exited child. status: exit code (>= 0) or -signal.
PLX_API int plx_pm_wait(void* h, int timeout_ms, int* out_pid, int* out_status) {
  Monitor* m = static_cast<Monitor*>(h);
  for (;;) {
    epoll_event ev{};
    int n = epoll_wait(m->ep, &ev, 1, timeout_ms);
    if (n < 0) {
      if (errno == EINTR) continue;
      return -errno;
    }
    if (n == 0) return 0;
    if (ev.data.fd == m->wake_fd) {
      uint64_t v;
      while (read(m->wake_fd, &v, sizeof(v)) > 0) {
      }
      return 2;
    }
    pid_t pid;
    {
      std::lock_guard<std::mutex> lk(m->mu);
      auto it = m->fd_to_pid.find(ev.data.fd);
      if (it == m->fd_to_pid.end()) continue;
      pid = it->second;
    }
    int st = 0;
    pid_t r = waitpid(pid, &st, WNOHANG);
    if (r == 0) continue;  // spurious
    // Forget the pidfd BEFORE closing it: once closed, its number can be handed to the next pidfd_open on the
    // spawning thread, and erasing fd_to_pid[fd] after that would drop the NEW child's entry -- its exit would
    // then never be reaped (level-triggered epoll keeps reporting an fd this loop no longer knows).  Found as an
    // intermittent timeout of tests/native/procmon_stress.cpp under TSan (slow spawns widen the window).
    {
      std::lock_guard<std::mutex> lk(m->mu);
      m->fd_to_pid.erase(ev.data.fd);
      m->pid_to_fd.erase(pid);
    }
    epoll_ctl(m->ep, EPOLL_CTL_DEL, ev.data.fd, nullptr);
    close(ev.data.fd);
    *out_pid = (int)pid;
    if (r < 0)
      *out_status = -255;
    else if (WIFEXITED(st))
      *out_status = WEXITSTATUS(st);
    else if (WIFSIGNALED(st))
      *out_status = -WTERMSIG(st);
    else
      *out_status = -255;
    return 1;
  }
}

PLX_API void plx_pm_wake(void* h) {
  Monitor* m = static_cast<Monitor*>(h);
  uint64_t one = 1;
  ssize_t w = write(m->wake_fd, &one, sizeof(one));
  (void)w;
}

PLX_API int plx_pm_signal(void* h, int pid, int sig, int group) {
  (void)h;
  int rc = group ? killpg((pid_t)pid, sig) : kill((pid_t)pid, sig);
  return rc == 0 ? 0 : errno;
}

PLX_API int plx_pm_count(void* h) {
  Monitor* m = static_cast<Monitor*>(h);
  std::lock_guard<std::mutex> lk(m->mu);
  return (int)m->pid_to_fd.size();
}

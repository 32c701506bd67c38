// Host-side stress test of the polyflow process supervisor (polyaxon_amd/csrc/procmon.cpp), built with
// -fsanitize=address,undefined and, separately, -fsanitize=thread by tests/test_sanitizers.py
// (the reference has no race detection; this is the native scheduler core's).
//
// One thread spawns N short-lived children with known exit codes (some killed by a signal), one thread reaps
// them through plx_pm_wait, one thread hammers plx_pm_wake / plx_pm_count concurrently.  Every child must be
// reaped exactly once with its exact status, and the monitor must end empty.
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

#include <atomic>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../polyaxon_amd/csrc/procmon.cpp"

extern char** environ;

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 200;
  void* h = plx_pm_create();
  if (!h) {
    fprintf(stderr, "create failed\n");
    return 2;
  }
  std::mutex mu;
  std::map<int, int> expected;  // pid -> expected status
  std::atomic<int> spawned{0};
  std::atomic<bool> done{false};

  std::thread spawner([&] {
    for (int i = 0; i < n; ++i) {
      std::string code = "exit " + std::to_string(i % 7);
      const bool killed = i % 11 == 0;
      if (killed) code = "kill -TERM $$; sleep 5";
      char* args[] = {(char*)"/bin/sh", (char*)"-c", (char*)code.c_str(), nullptr};
      int pid = 0;
      std::lock_guard<std::mutex> lk(mu);  // record before the reaper can see the exit
      const int rc = plx_pm_spawn(h, args, environ, nullptr, nullptr, &pid);
      if (rc != 0) {
        fprintf(stderr, "spawn %d failed: %d\n", i, rc);
        exit(3);
      }
      expected[pid] = killed ? -SIGTERM : i % 7;
      spawned.fetch_add(1);
    }
  });
  std::thread noise([&] {
    while (!done.load()) {
      plx_pm_wake(h);
      (void)plx_pm_count(h);
      usleep(50);
    }
  });
  int reaped = 0, bad = 0;
  std::map<int, int> seen;
  while (reaped < n) {
    int pid = 0, st = 0;
    const int r = plx_pm_wait(h, 2000, &pid, &st);
    if (r == 1) {
      std::lock_guard<std::mutex> lk(mu);
      if (seen.count(pid) || !expected.count(pid) || expected[pid] != st) {
        fprintf(stderr, "pid %d status %d expected %d seen %d\n", pid, st, expected.count(pid) ? expected[pid] : 999,
                (int)seen.count(pid));
        ++bad;
      }
      seen[pid] = st;
      ++reaped;
    } else if (r == 0 && spawned.load() == n) {
      fprintf(stderr, "timeout with %d/%d reaped\n", reaped, n);
      ++bad;
      break;
    } else if (r < 0) {
      fprintf(stderr, "wait error %d\n", r);
      ++bad;
      break;
    }
  }
  spawner.join();
  done.store(true);
  noise.join();
  const int left = plx_pm_count(h);
  plx_pm_destroy(h);
  printf("spawned %d reaped %d bad %d left %d\n", spawned.load(), reaped, bad, left);
  return (bad == 0 && left == 0 && reaped == n) ? 0 : 1;
}

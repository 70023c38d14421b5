// The mark a process leaves for the node daemon once its waves are countable
// on some GPUs (CounterVisibility.h): a 4 KiB memfd mapping named
// "dynolog-countable:<kfd gpu_id>,<kfd gpu_id>,...", which shows in
// /proc/<pid>/maps as "/memfd:dynolog-countable:...".  It exists exactly as
// long as the process and names exactly the GPUs whose device counting
// service the process configured (libdyno_countable.so, or the agent's
// preinit in libdyno_rocprof.so); merely loading a library proves nothing.
#pragma once

#include <sys/mman.h>
#include <unistd.h>

#include <cstdint>
#include <string>
#include <vector>

inline constexpr char kDynoCountableMark[] = "dynolog-countable:";

inline bool dynoMarkCountable(const std::vector<uint64_t>& gpuIds) {
  if (gpuIds.empty()) return false;
  std::string name = kDynoCountableMark;
  for (size_t i = 0; i < gpuIds.size(); ++i) name += (i ? "," : "") + std::to_string(gpuIds[i]);
  if (name.size() > 240) name.resize(240);  // memfd names are short; 8 GPUs fit easily
  const int fd = memfd_create(name.c_str(), MFD_CLOEXEC);
  if (fd < 0) return false;
  bool ok = ftruncate(fd, 4096) == 0;
  if (ok) ok = mmap(nullptr, 4096, PROT_READ, MAP_SHARED, fd, 0) != MAP_FAILED;  // kept for the process's life
  close(fd);
  return ok;
}

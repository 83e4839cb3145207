// Read-only mmap of a whole file (shared by the text loader and the binary CSR cache).
#pragma once
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <stdexcept>
#include <string>

namespace fm {

struct MappedFile {
  const char* data = nullptr;
  size_t size = 0;
  explicit MappedFile(const std::string& path, int advice = MADV_SEQUENTIAL) {
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("cannot open " + path + ": " + std::strerror(errno));
    struct stat st {};
    if (::fstat(fd, &st) != 0) {
      ::close(fd);
      throw std::runtime_error("cannot stat " + path);
    }
    size = static_cast<size_t>(st.st_size);
    if (size > 0) {
      void* p = ::mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
      if (p == MAP_FAILED) {
        ::close(fd);
        throw std::runtime_error("cannot map " + path);
      }
      ::madvise(p, size, advice);
      data = static_cast<const char*>(p);
    }
    ::close(fd);
  }
  ~MappedFile() {
    if (data) ::munmap(const_cast<char*>(data), size);
  }
  MappedFile(const MappedFile&) = delete;
  MappedFile& operator=(const MappedFile&) = delete;
};

}  // namespace fm

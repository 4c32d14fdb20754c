// Single-writer / multi-reader shared-memory broadcast channel for TP step metadata.
//
// The reference has no multi-GPU path at all (no collectives, TP cannot be
// configured - llm/config/llama-3.1-8b.yaml:2,8 is never read).  The MI355X build runs one
// process per GPU; rank 0 owns the scheduler and block manager and must hand every TP
// worker the same packed int32 step descriptor before all ranks launch
// the identical kernel / RCCL sequence.  Doing that through RCCL would leave an idle
// worker parked inside a collective (and the process-group watchdog kills it after its
// timeout); a POSIX shared-memory mailbox costs ~1-2 us on one node, never times out while
// the server is idle, and keeps the GPU queues free of spinning kernels.
//
// Layout: [Header][slot 0][slot 1].  The writer publishes message `seq` into slot seq&1
// after every reader has acknowledged message seq-1 (so the slot it overwrites - seq-2's -
// is dead), then stores `seq` with release ordering.  Readers spin briefly, then back off
// with short sleeps, copy the slot out and store their ack (release).
//
// Rank liveness (SURVEY §5.3 "TP-rank liveness"): the header records the writer's pid and
// every attached reader's pid.  A writer waiting for acks checks its readers' pids while it
// backs off and fails the publish naming the dead rank; a reader can ask whether the writer
// is still alive between timed receives, so a TP worker exits when rank 0 dies instead of
// spinning forever.
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

namespace py = pybind11;

namespace {

constexpr int kMaxReaders = 64;
constexpr uint64_t kMagic = 0x4154544153484d32ull;  // "ATTASHM2"

struct alignas(64) Header {
  uint64_t magic;
  uint32_t capacity;   // int32 words per slot
  uint32_t n_readers;
  int32_t writer_pid;
  // CLOCK_MONOTONIC (system-wide) deadline by which every reader must have registered; a
  // reader still unregistered after it counts as dead (e.g. a worker that died while
  // loading weights, before register_reader).  0 = no deadline.
  int64_t register_deadline_ns;
  alignas(64) std::atomic<uint64_t> seq;
  alignas(64) std::atomic<uint32_t> closed;
  alignas(64) std::atomic<uint64_t> acks[kMaxReaders];
  std::atomic<int32_t> reader_pids[kMaxReaders];  // 0 = not attached yet
  uint32_t slot_words[2];
};

// true unless `pid` provably no longer exists (EPERM: alive but not ours)
inline bool pid_alive(int32_t pid) {
  return pid <= 0 || kill(static_cast<pid_t>(pid), 0) == 0 || errno != ESRCH;
}

inline int64_t mono_ns() {
  timespec ts{};
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000ll + ts.tv_nsec;
}

inline void cpu_relax() { __builtin_ia32_pause(); }

inline void backoff(uint64_t& spins) {
  ++spins;
  if (spins < 20000) {
    cpu_relax();
  } else {
    // idle server: ~50-200 us sleeps keep an idle worker at a few % of one core
    timespec ts{0, spins < 200000 ? 20000L : 200000L};
    nanosleep(&ts, nullptr);
  }
}

class ShmChannel {
 public:
  ShmChannel(const std::string& name, int64_t capacity_words, int n_readers, bool create,
             double register_timeout_s)
      : name_(name.empty() || name[0] != '/' ? "/" + name : name), owner_(create) {
    if (n_readers < 0 || n_readers > kMaxReaders) throw std::invalid_argument("n_readers");
    int fd = -1;
    if (create) {
      if (capacity_words <= 0) throw std::invalid_argument("capacity_words");
      shm_unlink(name_.c_str());
      fd = shm_open(name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm_open(create) failed: " + name_);
      bytes_ = sizeof(Header) + 2 * static_cast<size_t>(capacity_words) * 4;
      if (ftruncate(fd, static_cast<off_t>(bytes_)) != 0) {
        close(fd);
        throw std::runtime_error("ftruncate failed");
      }
    } else {
      fd = shm_open(name_.c_str(), O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm_open(attach) failed: " + name_);
      struct stat st{};
      fstat(fd, &st);
      bytes_ = static_cast<size_t>(st.st_size);
      if (bytes_ < sizeof(Header)) {
        close(fd);
        throw std::runtime_error("shm segment too small");
      }
    }
    void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("mmap failed");
    hdr_ = static_cast<Header*>(p);
    if (create) {
      hdr_->capacity = static_cast<uint32_t>(capacity_words);
      hdr_->n_readers = static_cast<uint32_t>(n_readers);
      hdr_->writer_pid = static_cast<int32_t>(getpid());
      hdr_->register_deadline_ns =
          register_timeout_s > 0
              ? mono_ns() + static_cast<int64_t>(register_timeout_s * 1e9)
              : 0;
      for (auto& r : hdr_->reader_pids) r.store(0, std::memory_order_relaxed);
      hdr_->seq.store(0, std::memory_order_relaxed);
      hdr_->closed.store(0, std::memory_order_relaxed);
      for (auto& a : hdr_->acks) a.store(0, std::memory_order_relaxed);
      std::atomic_thread_fence(std::memory_order_release);
      hdr_->magic = kMagic;
    } else if (hdr_->magic != kMagic) {
      throw std::runtime_error("shm channel not initialised: " + name_);
    }
    slots_ = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(p) + sizeof(Header));
  }

  ~ShmChannel() {
    if (hdr_) munmap(hdr_, bytes_);
    if (owner_) shm_unlink(name_.c_str());
  }

  int64_t capacity() const { return hdr_->capacity; }
  int n_readers() const { return static_cast<int>(hdr_->n_readers); }
  uint64_t seq() const { return hdr_->seq.load(std::memory_order_acquire); }
  bool closed() const { return hdr_->closed.load(std::memory_order_acquire) != 0; }
  bool writer_alive() const { return pid_alive(hdr_->writer_pid); }

  // A reader announces its pid so the writer can tell a dead rank from a slow one.
  void register_reader(int reader) {
    check_reader(reader);
    hdr_->reader_pids[reader].store(static_cast<int32_t>(getpid()), std::memory_order_release);
  }

  // Reader ids whose registered process no longer exists, or that never registered before
  // the registration deadline.
  py::list dead_readers() const {
    py::list out;
    for (uint32_t r = 0; r < hdr_->n_readers; ++r)
      if (reader_dead(r)) out.append(r);
    return out;
  }

  // Reader ids that have not registered yet.
  py::list unregistered_readers() const {
    py::list out;
    for (uint32_t r = 0; r < hdr_->n_readers; ++r)
      if (hdr_->reader_pids[r].load(std::memory_order_acquire) == 0) out.append(r);
    return out;
  }

  // Publish one message; blocks (GIL released) until the slot is free.  Returns its seq.
  uint64_t publish(py::array_t<int32_t, py::array::c_style | py::array::forcecast> a,
                   double timeout_s) {
    const int64_t n = a.size();
    if (n > static_cast<int64_t>(hdr_->capacity)) throw std::length_error("message too large");
    const int32_t* src = a.data();
    const uint64_t next = hdr_->seq.load(std::memory_order_relaxed) + 1;
    int rc = 0;
    {
      py::gil_scoped_release nogil;
      rc = wait_acks(next - 1, timeout_s);
      if (rc == 0) {
        int32_t* dst = slots_ + static_cast<size_t>(next & 1) * hdr_->capacity;
        std::memcpy(dst, src, static_cast<size_t>(n) * 4);
        hdr_->slot_words[next & 1] = static_cast<uint32_t>(n);
        hdr_->seq.store(next, std::memory_order_release);
      }
    }
    if (rc > 0)
      throw std::runtime_error("shm channel: reader " + std::to_string(rc - 1) +
                               " (TP rank " + std::to_string(rc) + ") died");
    if (rc < 0) throw std::runtime_error("shm channel: readers did not acknowledge in time");
    return next;
  }

  // Wait for a message newer than `last_seq`; returns (seq, int32 array) or None when the
  // channel was closed or the timeout (<0: forever) expired.
  py::object receive(int reader, uint64_t last_seq, double timeout_s) {
    check_reader(reader);
    uint64_t s = 0;
    bool got = false;
    py::array_t<int32_t> out;
    {
      py::gil_scoped_release nogil;
      const auto t0 = std::chrono::steady_clock::now();
      uint64_t spins = 0;
      for (;;) {
        s = hdr_->seq.load(std::memory_order_acquire);
        if (s > last_seq) {
          got = true;
          break;
        }
        if (hdr_->closed.load(std::memory_order_acquire)) break;
        if (timeout_s >= 0 && (spins & 1023) == 0) {
          const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0)
                                .count();
          if (el > timeout_s) break;
        }
        backoff(spins);
      }
    }
    if (!got) return py::none();
    if (s > last_seq + 1)  // the writer never runs more than one message ahead of any reader
      throw std::runtime_error("shm channel: reader fell behind");
    const uint32_t n = hdr_->slot_words[s & 1];
    out = py::array_t<int32_t>(n);
    std::memcpy(out.mutable_data(), slots_ + static_cast<size_t>(s & 1) * hdr_->capacity,
                static_cast<size_t>(n) * 4);
    hdr_->acks[reader].store(s, std::memory_order_release);
    return py::make_tuple(s, out);
  }

  void close_channel() { hdr_->closed.store(1, std::memory_order_release); }

 private:
  void check_reader(int reader) const {
    if (reader < 0 || reader >= static_cast<int>(hdr_->n_readers))
      throw std::out_of_range("reader id");
  }

  bool reader_dead(uint32_t r) const {
    const int32_t pid = hdr_->reader_pids[r].load(std::memory_order_acquire);
    if (pid == 0)
      return hdr_->register_deadline_ns > 0 && mono_ns() > hdr_->register_deadline_ns;
    return !pid_alive(pid);
  }

  // 0: every reader acknowledged `target`; -1: timeout; r + 1: reader r's process is gone.
  int wait_acks(uint64_t target, double timeout_s) {
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t spins = 0;
    for (uint32_t r = 0; r < hdr_->n_readers; ++r) {
      while (hdr_->acks[r].load(std::memory_order_acquire) < target) {
        if ((spins & 1023) == 1023) {
          if (reader_dead(r)) return static_cast<int>(r) + 1;
          if (timeout_s >= 0) {
            const double el =
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (el > timeout_s) return -1;
          }
        }
        backoff(spins);
      }
    }
    return 0;
  }

  std::string name_;
  bool owner_;
  size_t bytes_ = 0;
  Header* hdr_ = nullptr;
  int32_t* slots_ = nullptr;
};

}  // namespace

void register_shm_channel(py::module_& m) {
  py::class_<ShmChannel>(m, "ShmChannel")
      .def(py::init<const std::string&, int64_t, int, bool, double>(), py::arg("name"),
           py::arg("capacity_words") = 0, py::arg("n_readers") = 0, py::arg("create") = false,
           py::arg("register_timeout_s") = 0.0)
      .def_property_readonly("capacity", &ShmChannel::capacity)
      .def_property_readonly("n_readers", &ShmChannel::n_readers)
      .def_property_readonly("seq", &ShmChannel::seq)
      .def_property_readonly("closed", &ShmChannel::closed)
      .def_property_readonly("writer_alive", &ShmChannel::writer_alive)
      .def("register_reader", &ShmChannel::register_reader, py::arg("reader"))
      .def("dead_readers", &ShmChannel::dead_readers)
      .def("unregistered_readers", &ShmChannel::unregistered_readers)
      .def("publish", &ShmChannel::publish, py::arg("data"), py::arg("timeout_s") = -1.0)
      .def("receive", &ShmChannel::receive, py::arg("reader"), py::arg("last_seq"),
           py::arg("timeout_s") = -1.0)
      .def("close", &ShmChannel::close_channel);
}

// host_pool.h -- a small worker pool for the host-side loops of the encoder
// (rate control, Tier-2 simulation): the reference runs its PCRD bisection
// serially on one thread per tile (TileProcessor.cpp:371-667); here each
// bisection step's per-code-block and per-precinct work is spread over the
// host cores, so rate control stays off the critical path of a frame whose
// Tier-1 took a few ms on the GPU.  One process-wide pool; the calling thread
// works on its own loop too, so concurrent callers (frames in flight on other
// threads) never wait for an idle worker.
#pragma once
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace grkgpu {

class HostPool {
public:
    static HostPool &get() {
        static HostPool p;
        return p;
    }

    size_t workers() const { return threads_.size(); }

    // f(begin, end) over [0, n) in chunks of `grain` items, on the pool and
    // the caller; returns when every chunk has run.  The chunks are disjoint,
    // so f may write per-item results without synchronisation.
    void parallel_for(size_t n, size_t grain, const std::function<void(size_t, size_t)> &f) {
        if (!n) return;
        grain = std::max<size_t>(grain, 1);
        const size_t nchunks = (n + grain - 1) / grain;
        if (nchunks == 1 || threads_.empty()) {
            f(0, n);
            return;
        }
        Job j;
        j.f = &f;
        j.n = n;
        j.grain = grain;
        j.nchunks = nchunks;
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_.push_back(&j);
        }
        cv_.notify_all();
        run(j);
        // leave the queue, then wait for the workers still inside this job
        {
            std::unique_lock<std::mutex> lk(mu_);
            auto it = std::find(q_.begin(), q_.end(), &j);
            if (it != q_.end()) q_.erase(it);
            done_cv_.wait(lk, [&] { return j.users == 0 && j.done.load() == j.nchunks; });
        }
    }

private:
    struct Job {
        const std::function<void(size_t, size_t)> *f = nullptr;
        size_t n = 0, grain = 1, nchunks = 0;
        std::atomic<size_t> next{0}, done{0};
        int users = 0;  // workers inside the job (guarded by mu_)
    };

    HostPool() {
        // GRKGPU_HOST_THREADS sets the pool size (the caller counts as one).
        // Default: half the CPUs this process may use -- its affinity mask,
        // or the cgroup's CPU quota when that is smaller (a GPU box: 16 of
        // 256), at most 16 -- since the frames in flight run their own host
        // work on their own threads beside the pool, and threads beyond the
        // quota get the whole process throttled.  Measured on one box, pool
        // of 16 / 8 (profiles/r05/host_pool_ab.txt): DCI 4K cinema batch
        // 2029-2228 -> 2464-2533 Mpixels/s, the 8K batch 3526 / 3555 ->
        // 3546 / 3622, the C4 tile shard 2278 / 2273 -> 2215 / 2260.
        size_t n = std::thread::hardware_concurrency();
        {
            cpu_set_t set;
            if (sched_getaffinity(0, sizeof(set), &set) == 0 && CPU_COUNT(&set) > 0) n = (size_t)CPU_COUNT(&set);
        }
        const size_t quota = cgroup_cpus();
        if (quota && quota < n) n = quota;
        n = std::max<size_t>(std::min<size_t>(n, 16) / 2, 1);
        if (const char *e = getenv("GRKGPU_HOST_THREADS")) n = std::min<size_t>(std::max(atoi(e), 1), 16);
        for (size_t i = 1; i < n; ++i) threads_.emplace_back([this] { loop(); });
    }
    // CPUs of the cgroup's quota, 0 if none: the process's own cgroup from
    // /proc/self/cgroup (v2 "0::/path" -> cpu.max "quota period"; v1 the cpu
    // controller's line -> cfs_quota_us / cfs_period_us), each directory from
    // it up to the mount root, the smallest quota found (a parent's limit
    // binds too); a namespaced cgroup whose path is "/" reads the root files.
    static size_t cgroup_cpus() {
        std::string v2, v1;
        if (FILE *f = fopen("/proc/self/cgroup", "r")) {
            char line[4096];
            while (fgets(line, sizeof(line), f)) {
                std::string l(line);
                while (!l.empty() && (l.back() == '\n' || l.back() == '\r')) l.pop_back();
                const size_t c1 = l.find(':'), c2 = c1 == std::string::npos ? c1 : l.find(':', c1 + 1);
                if (c2 == std::string::npos) continue;
                const std::string ctl = l.substr(c1 + 1, c2 - c1 - 1), path = l.substr(c2 + 1);
                if (l.compare(0, c1, "0") == 0 && ctl.empty()) v2 = path;
                else if (("," + ctl + ",").find(",cpu,") != std::string::npos) v1 = path;
            }
            fclose(f);
        }
        size_t best = 0;
        auto take = [&best](unsigned long long quota, unsigned long long period) {
            if (!period) return;
            const size_t n = (size_t)((quota + period - 1) / period);
            if (n && (!best || n < best)) best = n;
        };
        // each directory from `path` up to the root of `mount`
        auto walk = [](const std::string &mount, std::string path, const auto &fn) {
            for (;;) {
                fn(mount + (path == "/" ? std::string() : path));
                if (path.empty() || path == "/") break;
                const size_t k = path.rfind('/');
                path = k == 0 || k == std::string::npos ? "/" : path.substr(0, k);
            }
        };
        walk("/sys/fs/cgroup", v2.empty() ? "/" : v2, [&](const std::string &d) {
            if (FILE *f = fopen((d + "/cpu.max").c_str(), "r")) {
                char q[32] = {0};
                unsigned long long period = 0;
                if (fscanf(f, "%31s %llu", q, &period) == 2 && strcmp(q, "max") != 0)
                    take(strtoull(q, nullptr, 10), period);
                fclose(f);
            }
        });
        walk("/sys/fs/cgroup/cpu", v1.empty() ? "/" : v1, [&](const std::string &d) {
            long long q = -1;
            unsigned long long period = 0;
            if (FILE *f = fopen((d + "/cpu.cfs_quota_us").c_str(), "r")) {
                if (fscanf(f, "%lld", &q) != 1) q = -1;
                fclose(f);
            }
            if (q <= 0) return;
            if (FILE *g = fopen((d + "/cpu.cfs_period_us").c_str(), "r")) {
                if (fscanf(g, "%llu", &period) == 1) take((unsigned long long)q, period);
                fclose(g);
            }
        });
        return best;
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : threads_) t.join();
    }

    void run(Job &j) {
        size_t c;
        while ((c = j.next.fetch_add(1)) < j.nchunks) {
            const size_t b = c * j.grain;
            (*j.f)(b, std::min(j.n, b + j.grain));
            j.done.fetch_add(1);
        }
    }

    void loop() {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
            if (stop_) return;
            Job *j = q_.front();
            if (j->next.load() >= j->nchunks) {  // exhausted: drop it, its caller finishes it
                q_.pop_front();
                continue;
            }
            ++j->users;
            lk.unlock();
            run(*j);
            lk.lock();
            if (--j->users == 0) done_cv_.notify_all();
        }
    }

    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::deque<Job *> q_;
    std::vector<std::thread> threads_;
    bool stop_ = false;
};

inline void host_parallel_for(size_t n, size_t grain, const std::function<void(size_t, size_t)> &f) {
    HostPool::get().parallel_for(n, grain, f);
}

}  // namespace grkgpu

// vcfc_queue.h -- the hand-off queue between the host pipeline stages of the
// drivers (vcfc_ingest_driver.h, vcfc_decode_driver.h).
#pragma once
#include <condition_variable>
#include <deque>
#include <mutex>

namespace vcfc_q {

template <class T>
struct Queue {
    std::mutex m;
    std::condition_variable cv;
    std::deque<T> q;
    bool closed = false;
    void put(T v) {
        std::lock_guard<std::mutex> g(m);
        q.push_back(std::move(v));
        cv.notify_all();
    }
    bool get(T &v) {   // false once closed and empty
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, [&] { return !q.empty() || closed; });
        if (q.empty()) return false;
        v = std::move(q.front());
        q.pop_front();
        return true;
    }
    void close() {
        std::lock_guard<std::mutex> g(m);
        closed = true;
        cv.notify_all();
    }
};

}  // namespace vcfc_q

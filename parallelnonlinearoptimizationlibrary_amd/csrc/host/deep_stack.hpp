// deep_stack.hpp -- run a solver body on a thread with a large stack.
//
// The bounded BFGS classes re-optimise the reduced problem recursively from
// boundaryAssessment (BFGS_bnd_linesearch.cpp:620): one level deeper per coordinate that
// reaches a bound, which is about 11k levels at n = 16384 (SURVEY 8(d) cfg 5) -- far past a
// default 8 MiB thread stack.  The body runs on a joined worker thread whose stack is reserved
// (not committed) up front; exceptions are carried back to the caller.
#pragma once

#include <pthread.h>

#include <exception>
#include <utility>

namespace pnol {

template <class F>
void run_deep(F&& body, size_t stack_bytes = (size_t)1 << 30) {
    struct Job {
        F* f;
        std::exception_ptr err;
    } job{&body, nullptr};
    pthread_attr_t attr;
    pthread_t th;
    bool started = false;
    if (pthread_attr_init(&attr) == 0) {
        if (pthread_attr_setstacksize(&attr, stack_bytes) == 0)
            started = pthread_create(&th, &attr,
                                     +[](void* a) -> void* {
                                         Job* j = static_cast<Job*>(a);
                                         try {
                                             (*j->f)();
                                         } catch (...) {
                                             j->err = std::current_exception();
                                         }
                                         return nullptr;
                                     },
                                     &job) == 0;
        pthread_attr_destroy(&attr);
    }
    if (!started) {   // no worker thread: run in place (shallow problems still work)
        body();
        return;
    }
    pthread_join(th, nullptr);
    if (job.err) std::rethrow_exception(job.err);
}

}  // namespace pnol

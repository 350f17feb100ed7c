// mc_setorder.inl — reference-exact orders of the clustered containers, restated natively (host
// code; included by mc_api.hip).
//
// The reference's final objects are Python containers whose ITERATION ORDER its exports follow:
//   * networkx connected_components (graph/iterative_clustering.py:7) yields every component as the
//     `seen` set of _plain_bfs (networkx 3.x: BFS from the smallest unseen node, `seen.add` in
//     discovery order, neighbours ascending because from_numpy_array inserts the row-major edges of
//     A, :30-32);
//   * Node.create_node_from_list (graph/node.py:24-37) walks that set: mask_list += member.mask_list,
//     point_ids = point_ids.union(member.point_ids), son_node_info.add(member.node_info);
//   * the level-0 point sets are set(ndarray of ascending scene ids) (utils/mask_backprojection.py:
//     139-148), aliased by init_nodes (graph/construction.py:66-78);
//   * post_process reads list(point_ids) (graph/node.py:45, utils/post_process.py:185) and mask_list.
// CPython's set (Objects/setobject.c) fixes those orders as a function of the keys' hashes (an int,
// np.int64 included, hashes to itself) and the insertion history.  PySet below replays exactly that
// history on int keys: open addressing from hash & mask, up to 9 linear probes (only when they do not
// wrap), then perturbed probing i = 5i + 1 + (perturb >>= 5); a table resized when fill * 5 >= mask * 3
// after an insert (to the smallest power of two > 4 * used, > 2 * used above 50000 entries; the old
// entries re-inserted in slot order); union = copy (a new set merged from the left operand) + merge of
// the right operand with one up-front resize when (fill + other.used) * 5 >= mask * 3 (to > 2 * (used +
// other.used)); a merge into an empty set copies the table verbatim when the masks agree, else
// re-inserts in slot order.  The reference never removes from these sets, so no table ever holds a
// dummy.  Pinned against the running interpreter (tests/test_setorder_cpu.py: random histories and the
// reference's own exports, tests/golden/e2e_pp_small_*).
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <system_error>
#include <thread>
#include <pthread.h>
#include <vector>

#include <unistd.h>

namespace mcso {

constexpr size_t kLinearProbes = 9;
constexpr int kPerturbShift = 5;
constexpr size_t kMinSize = 8;

struct PySet {
    std::vector<int32_t> t;  // key, or -1 = empty slot
    size_t mask = kMinSize - 1;
    size_t used = 0;         // == fill (no dummies)
    PySet() : t(kMinSize, -1) {}
};

// Tables are recycled per thread (by power-of-two size, up to 8 MB held per thread): a replay makes
// and drops tens of millions of slots, and fresh large blocks cost page faults and, when returned to
// the OS from a many-threaded process, TLB shootdowns.
struct TablePool {
    std::vector<std::vector<int32_t>> bins[40];
    size_t bytes = 0;
};
inline TablePool &table_pool()
{
    thread_local TablePool p;
    return p;
}
inline int log2_pow2(size_t n)
{
    int b = 0;
    while ((static_cast<size_t>(1) << b) < n) b++;
    return b;
}
constexpr size_t kPoolMinSlots = 256;
inline std::vector<int32_t> take_table(size_t ns)
{
    if (ns >= kPoolMinSlots) {
        TablePool &p = table_pool();
        auto &bin = p.bins[log2_pow2(ns)];
        if (!bin.empty()) {
            std::vector<int32_t> v = std::move(bin.back());
            bin.pop_back();
            p.bytes -= ns * sizeof(int32_t);
            std::fill(v.begin(), v.end(), -1);
            return v;
        }
    }
    return std::vector<int32_t>(ns, -1);
}
inline void give_table(std::vector<int32_t> &&v)
{
    const size_t ns = v.size();
    if (ns < kPoolMinSlots || (ns & (ns - 1))) return;
    TablePool &p = table_pool();
    if (p.bytes + ns * sizeof(int32_t) > (static_cast<size_t>(8) << 20)) return;
    p.bins[log2_pow2(ns)].push_back(std::move(v));
    p.bytes += ns * sizeof(int32_t);
}

// set_insert_clean: the first empty slot of key's probe sequence (no key comparisons)
inline void insert_clean(int32_t *tab, size_t mask, int32_t key)
{
    size_t perturb = static_cast<size_t>(key);
    size_t i = static_cast<size_t>(key) & mask;
    while (true) {
        if (tab[i] < 0) {
            tab[i] = key;
            return;
        }
        if (i + kLinearProbes <= mask) {
            for (size_t j = 1; j <= kLinearProbes; j++)
                if (tab[i + j] < 0) {
                    tab[i + j] = key;
                    return;
                }
        }
        perturb >>= kPerturbShift;
        i = (i * 5 + 1 + perturb) & mask;
    }
}

// set_table_resize(so, minused)
inline void resize(PySet &s, size_t minused)
{
    size_t ns = kMinSize;
    while (ns <= minused) ns <<= 1;
    if (ns == kMinSize && s.mask == kMinSize - 1) return;  // the small table, no dummies: nothing to do
    std::vector<int32_t> nt = take_table(ns);
    for (int32_t k : s.t)
        if (k >= 0) insert_clean(nt.data(), ns - 1, k);
    s.t.swap(nt);
    s.mask = ns - 1;
    give_table(std::move(nt));
}

// set_add_entry (keys are distinct ints: an equal hash is an equal key)
inline void add(PySet &s, int32_t key)
{
    int32_t *tab = s.t.data();
    const size_t mask = s.mask;
    size_t i = static_cast<size_t>(key) & mask;
    size_t at;
    if (tab[i] < 0) {
        at = i;
    } else {
        size_t perturb = static_cast<size_t>(key);
        while (true) {
            if (tab[i] == key) return;
            if (i + kLinearProbes <= mask) {
                for (size_t j = 1; j <= kLinearProbes; j++) {
                    if (tab[i + j] < 0) {
                        at = i + j;
                        goto found;
                    }
                    if (tab[i + j] == key) return;
                }
            }
            perturb >>= kPerturbShift;
            i = (i * 5 + 1 + perturb) & mask;
            if (tab[i] < 0) {
                at = i;
                goto found;
            }
        }
    }
found:
    tab[at] = key;
    s.used++;
    if (s.used * 5 < mask * 3) return;
    resize(s, s.used > 50000 ? s.used * 2 : s.used * 4);
}

// set_merge(so, other)
inline void merge(PySet &s, const PySet &o)
{
    if (o.used == 0) return;
    if ((s.used + o.used) * 5 >= s.mask * 3) resize(s, (s.used + o.used) * 2);
    if (s.used == 0) {
        if (s.mask == o.mask) {
            s.t = o.t;  // verbatim copy
        } else {
            for (int32_t k : o.t)
                if (k >= 0) insert_clean(s.t.data(), s.mask, k);
        }
        s.used = o.used;
        return;
    }
    for (int32_t k : o.t)
        if (k >= 0) add(s, k);
}

// merge() of a set the caller no longer needs: into an empty set whose mask (after the up-front
// resize) is the other's, the verbatim copy is the other's table itself
inline void merge_consume(PySet &s, PySet &&o)
{
    if (s.used == 0 && o.used != 0) {
        size_t ns = s.mask + 1;
        if ((s.used + o.used) * 5 >= s.mask * 3) {
            ns = kMinSize;
            while (ns <= (s.used + o.used) * 2) ns <<= 1;
            if (ns == kMinSize && s.mask == kMinSize - 1) ns = s.mask + 1;
        }
        if (ns - 1 == o.mask) {
            s = std::move(o);
            return;
        }
    }
    merge(s, o);
}

// a.union(b) when the caller no longer needs a: the copy step (make_new_set + set_merge into the
// empty set) keeps a's table when its mask is what the copy would size, else re-inserts in slot order
inline PySet union_consume(PySet &&a, PySet &&b)
{
    PySet r;
    if (a.used) {
        size_t ns = kMinSize;
        if (a.used * 5 >= (kMinSize - 1) * 3)
            while (ns <= a.used * 2) ns <<= 1;
        if (ns - 1 == a.mask) {
            r = std::move(a);
        } else {
            r.t = take_table(ns);
            r.mask = ns - 1;
            for (int32_t k : a.t)
                if (k >= 0) insert_clean(r.t.data(), r.mask, k);
            r.used = a.used;
            give_table(std::move(a.t));
        }
    }
    merge_consume(r, std::move(b));
    give_table(std::move(b.t));  // (empty when b's table moved into r)
    return r;
}

inline PySet union_consume(PySet &&a, const PySet &b)
{
    PySet r;
    if (a.used) {
        size_t ns = kMinSize;
        if (a.used * 5 >= (kMinSize - 1) * 3)
            while (ns <= a.used * 2) ns <<= 1;
        if (ns - 1 == a.mask) {
            r = std::move(a);
        } else {
            r.t = take_table(ns);
            r.mask = ns - 1;
            for (int32_t k : a.t)
                if (k >= 0) insert_clean(r.t.data(), r.mask, k);
            r.used = a.used;
            give_table(std::move(a.t));
        }
    }
    merge(r, b);
    return r;
}

// set(iterable): empty set, add in order
inline PySet from_sequence(const int32_t *v, int64_t n)
{
    PySet s;
    for (int64_t i = 0; i < n; i++) add(s, v[i]);
    return s;
}

// Workers kept for the whole replay (one set of threads instead of a spawn per level): run(fn) runs fn
// on every worker and the calling thread and returns when all are done.
class Pool {
  public:
    explicit Pool(int n) : n_(n)
    {
        for (int i = 1; i < n_; i++) th_.emplace_back([this] { loop(); });
    }
    ~Pool()
    {
        {
            std::lock_guard<std::mutex> g(mu_);
            quit_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    void run(const std::function<void()> &fn)
    {
        if (n_ == 1) return fn();
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = &fn;
            busy_ = n_ - 1;
            gen_++;
        }
        cv_.notify_all();
        fn();
        std::unique_lock<std::mutex> l(mu_);
        done_.wait(l, [this] { return busy_ == 0; });
        job_ = nullptr;
    }

  private:
    void loop()
    {
        unsigned seen = 0;
        while (true) {
            const std::function<void()> *job;
            {
                std::unique_lock<std::mutex> l(mu_);
                cv_.wait(l, [&] { return quit_ || gen_ != seen; });
                if (quit_) return;
                seen = gen_;
                job = job_;
            }
            (*job)();
            std::lock_guard<std::mutex> g(mu_);
            if (--busy_ == 0) done_.notify_one();
        }
    }
    int n_;
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void()> *job_ = nullptr;
    unsigned gen_ = 0;
    int busy_ = 0;
    bool quit_ = false;
};

// The workers of every replay in the process (created on first use, re-created when the thread count
// changes, left idle between calls): their per-thread table pools and malloc arenas stay warm.
// One replay step runs on them at a time.  MC_SETORDER_PERSIST=0: a pool per call instead.
class SharedPool {
  public:
    template <typename F>
    void run(int nth, F &&fn)
    {
        if (const char *e = getenv("MC_SETORDER_PERSIST"); e && atoi(e) == 0) {
            Pool p(nth);
            const std::function<void()> f = fn;
            p.run(f);
            return;
        }
        std::lock_guard<std::mutex> g(mu_);
        if (!pool_ || n_ != nth) {
            pool_.reset();
            pool_.reset(new Pool(nth));
            n_ = nth;
        }
        const std::function<void()> f = fn;
        pool_->run(f);
    }

  private:
    std::mutex mu_;
    std::unique_ptr<Pool> pool_;
    int n_ = 0;
};
// One per process.  A forked child inherits the parent's pool object (its n_ matching, its mutexes
// possibly held by parent threads) but none of its worker threads, so the child must start from a new
// pool: a pthread_atfork child handler (registered once, on first use) drops the inherited pool
// (leaked: joining threads that do not exist, or waiting on a mutex no thread will release, would
// hang) and re-initialises the creation mutex while the child still has only the forking thread.  The
// pid check stays as a second guard.
struct SharedPoolSlot {
    std::atomic<SharedPool *> p{nullptr};
    std::atomic<pid_t> owner{0};
    std::mutex mk;
};
inline SharedPoolSlot &shared_pool_slot()
{
    static SharedPoolSlot slot;
    return slot;
}
inline void shared_pool_atfork_child()
{
    SharedPoolSlot &sl = shared_pool_slot();
    sl.p.store(nullptr, std::memory_order_relaxed);
    sl.owner.store(0, std::memory_order_relaxed);
    new (&sl.mk) std::mutex;  // (one thread in the child: the inherited state may be locked)
}
inline SharedPool &shared_pool()
{
    static const bool registered = (pthread_atfork(nullptr, nullptr, shared_pool_atfork_child), true);
    (void)registered;
    SharedPoolSlot &sl = shared_pool_slot();
    const pid_t me = getpid();
    SharedPool *cur = sl.p.load(std::memory_order_acquire);
    if (cur && sl.owner.load(std::memory_order_acquire) == me) return *cur;
    std::lock_guard<std::mutex> g(sl.mk);
    cur = sl.p.load(std::memory_order_acquire);
    if (!cur || sl.owner.load(std::memory_order_acquire) != me) {
        cur = new SharedPool;  // never destroyed: idle workers end with the process
        sl.owner.store(me, std::memory_order_release);
        sl.p.store(cur, std::memory_order_release);
    }
    return *cur;
}

}  // namespace mcso

// Level-0 sets built ahead (mc_setorder_begin): a background thread makes every set(ascending ids)
// while the caller's device clustering runs; mc_setorder_finish replays the levels on them.
struct mc_setorder {
    int32_t n0 = 0;
    int nth = 1;
    std::vector<mcso::PySet> sets;
    std::thread th;
    int rc = MC_OK;
    bool consumed = false;
};

namespace mcso {

inline int threads_for(int32_t num_threads)
{
    // the caller's count, else MC_SETORDER_THREADS, else the host's threads capped by OMP_NUM_THREADS
    // (a process's CPU share: hardware_concurrency reports the whole machine).  On the C2 API path the
    // replay took 34 / 35 / 31 ms on average on 16 / 8 / 12 workers with +-8 ms between repeats
    // (profiles/r04/r4y_api_threads.txt): the full share stays the default
    int nth = num_threads;
    if (nth <= 0) {
        if (const char *e = getenv("MC_SETORDER_THREADS"); e && atoi(e) > 0) {
            nth = atoi(e);
        } else {
            nth = static_cast<int>(std::max(1u, std::thread::hardware_concurrency()));
            if (const char *o = getenv("OMP_NUM_THREADS")) nth = std::min(nth, std::max(1, atoi(o)));
        }
    }
    return std::max(1, std::min(nth, 64));
}

inline void build_level0(mc_setorder *h, const int64_t *node_start, const int64_t *node_len, const int32_t *pts)
{
    try {
        const int N0 = h->n0;
        std::atomic<int> next{0}, bad{0};
        auto work = [&]() {
            // chunks of 64 nodes: fewer shared-counter round trips than one node at a time; each node's
            // ids are checked by the worker that builds it (a negative id is not a scene point)
            for (int c = next.fetch_add(64); c < N0; c = next.fetch_add(64))
                for (int i = c; i < std::min(N0, c + 64); i++) {
                    const int32_t *q = pts + node_start[i];
                    bool ok = true;
                    for (int64_t k = 0; k < node_len[i]; k++) ok &= q[k] >= 0;
                    if (!ok) {
                        bad.store(1, std::memory_order_relaxed);
                        continue;
                    }
                    h->sets[i] = from_sequence(q, node_len[i]);
                }
        };
        shared_pool().run(h->nth, work);
        if (bad.load()) h->rc = MC_ERR_INVALID;
    } catch (const std::bad_alloc &) {
        h->rc = MC_ERR_HIP;
    }
}

}  // namespace mcso

extern "C" int mc_setorder_begin(int32_t num_nodes, const int64_t *node_start, const int64_t *node_len,
                                 const int32_t *pts, int32_t num_threads, int async_build, mc_setorder **out)
{
    if (!out || num_nodes < 0 || (num_nodes && (!node_start || !node_len))) return MC_ERR_INVALID;
    *out = nullptr;
    // O(num_nodes) range checks here; the ids themselves are checked by build_level0's workers (an
    // O(total points) loop on the caller's thread would sit on the critical path the async build hides)
    for (int i = 0; i < num_nodes; i++)
        if (node_start[i] < 0 || node_len[i] < 0 || (node_len[i] && !pts)) return MC_ERR_INVALID;
    try {
        auto *h = new mc_setorder;
        h->n0 = num_nodes;
        h->nth = mcso::threads_for(num_threads);
        h->sets.resize(static_cast<size_t>(num_nodes));
        if (async_build)
            h->th = std::thread(mcso::build_level0, h, node_start, node_len, pts);
        else
            mcso::build_level0(h, node_start, node_len, pts);
        *out = h;
        return MC_OK;
    } catch (const std::bad_alloc &) {
        return MC_ERR_HIP;
    } catch (const std::system_error &) {
        return MC_ERR_HIP;
    }
}

extern "C" void mc_setorder_free(mc_setorder *h)
{
    if (!h) return;
    if (h->th.joinable()) h->th.join();
    delete h;
}

extern "C" int mc_setorder_finish(mc_setorder *h, int32_t num_levels, const int32_t *level_sizes,
                                  const int64_t *edge_off, const int32_t *edge_a, const int32_t *edge_b,
                                  int32_t *num_objects, int64_t *obj_mask_off, int32_t *mask_order,
                                  int64_t *obj_pt_off, int32_t *obj_pts, int64_t *son_off, int32_t *son_order,
                                  int32_t *labels)
{
    using mcso::PySet;
    if (!h) return MC_ERR_INVALID;
    if (h->th.joinable()) h->th.join();
    if (h->rc != MC_OK) return h->rc;
    try {
        if (h->consumed || num_levels < 1 || !level_sizes || !edge_off || !num_objects || !obj_mask_off ||
            !mask_order || !obj_pt_off || !obj_pts || !son_off || !son_order)
            return MC_ERR_INVALID;
        const int T = num_levels;
        for (int t = 0; t < T; t++)
            if (level_sizes[t] < 0 || edge_off[t + 1] < edge_off[t]) return MC_ERR_INVALID;
        if (edge_off[0] != 0 || (edge_off[T] && (!edge_a || !edge_b))) return MC_ERR_INVALID;
        const int N0 = level_sizes[0];
        if (N0 != h->n0) return MC_ERR_INVALID;
        h->consumed = true;

        // per node of the current level: its mask order (level-0 indices) and point set
        std::vector<std::vector<int32_t>> morder(N0);
        for (int i = 0; i < N0; i++) morder[i].assign(1, i);
        std::vector<PySet> sets;
        sets.swap(h->sets);
        std::vector<int32_t> comp_off, comp_mem;  // the last level's components (member order)
        int64_t lab_base = 0;
        for (int t = 0; t < T; t++) {
            const int N = level_sizes[t];
            if (static_cast<int>(morder.size()) != N) return MC_ERR_INVALID;  // != components of t - 1
            // adjacency, ascending neighbours (from_numpy_array's row-major edge insertion)
            const int64_t e0 = edge_off[t], e1 = edge_off[t + 1];
            std::vector<int64_t> aoff(static_cast<size_t>(N) + 1, 0);
            for (int64_t e = e0; e < e1; e++) {
                const int a = edge_a[e], b = edge_b[e];
                if (a < 0 || b < 0 || a >= N || b >= N || a == b) return MC_ERR_INVALID;
                aoff[a + 1]++;
                aoff[b + 1]++;
            }
            for (int v = 0; v < N; v++) aoff[v + 1] += aoff[v];
            std::vector<int32_t> adj(static_cast<size_t>(aoff[N]));
            {
                std::vector<int64_t> cur(aoff.begin(), aoff.end() - 1);
                for (int64_t e = e0; e < e1; e++) {
                    adj[cur[edge_a[e]]++] = edge_b[e];
                    adj[cur[edge_b[e]]++] = edge_a[e];
                }
            }
            {  // edges sorted by (a, b) already give every list in ascending order
                bool sorted = true;
                for (int64_t e = e0 + 1; e < e1 && sorted; e++)
                    sorted = edge_a[e - 1] < edge_a[e] || (edge_a[e - 1] == edge_a[e] && edge_b[e - 1] < edge_b[e]);
                for (int64_t e = e0; e < e1 && sorted; e++) sorted = edge_a[e] < edge_b[e];
                if (!sorted)
                    for (int v = 0; v < N; v++) std::sort(adj.begin() + aoff[v], adj.begin() + aoff[v + 1]);
            }
            // components: _plain_bfs from every unseen node in order; `seen` is a set of node ints
            std::vector<int32_t> lab(static_cast<size_t>(N), -1);
            comp_off.assign(1, 0);
            comp_mem.clear();
            std::vector<int32_t> level, next;
            for (int v = 0; v < N; v++) {
                if (lab[v] >= 0) continue;
                const int k = static_cast<int>(comp_off.size()) - 1;
                if (aoff[v + 1] == aoff[v]) {  // an isolated node: {v}
                    lab[v] = k;
                    comp_mem.push_back(v);
                    comp_off.push_back(static_cast<int32_t>(comp_mem.size()));
                    continue;
                }
                PySet seen;
                mcso::add(seen, v);
                lab[v] = k;
                next.assign(1, v);
                while (!next.empty()) {
                    level.swap(next);
                    next.clear();
                    for (int32_t u : level)
                        for (int64_t j = aoff[u]; j < aoff[u + 1]; j++) {
                            const int32_t w = adj[j];
                            if (lab[w] < 0) {
                                lab[w] = k;
                                mcso::add(seen, w);
                                next.push_back(w);
                            } else if (lab[w] != k) {
                                return MC_ERR_INVALID;  // unreachable: BFS stays in its component
                            }
                        }
                }
                for (int32_t x : seen.t)
                    if (x >= 0) comp_mem.push_back(x);  // iteration order of the component set
                comp_off.push_back(static_cast<int32_t>(comp_mem.size()));
            }
            if (labels) std::copy(lab.begin(), lab.end(), labels + lab_base);
            lab_base += N;
            const int K = static_cast<int>(comp_off.size()) - 1;
            // create_node_from_list per component, in parallel over components; every set of this
            // level is read by exactly one component
            std::vector<std::vector<int32_t>> nmorder(K);
            std::vector<PySet> nsets(K);
            std::atomic<int> next_k{0};
            auto work = [&]() {
                for (int k = next_k++; k < K; k = next_k++) {
                    std::vector<int32_t> &mo = nmorder[k];
                    PySet acc;  // point_ids = set()
                    for (int32_t j = comp_off[k]; j < comp_off[k + 1]; j++) {
                        const int32_t m = comp_mem[j];
                        mo.insert(mo.end(), morder[m].begin(), morder[m].end());
                        acc = mcso::union_consume(std::move(acc), std::move(sets[m]));
                    }
                    nsets[k] = std::move(acc);
                }
            };
            mcso::shared_pool().run(h->nth, work);
            morder.swap(nmorder);
            sets.swap(nsets);
        }
        const int K = static_cast<int>(morder.size());
        *num_objects = K;
        obj_mask_off[0] = obj_pt_off[0] = son_off[0] = 0;
        int64_t mo = 0, po = 0;
        for (int k = 0; k < K; k++) {
            std::copy(morder[k].begin(), morder[k].end(), mask_order + mo);
            mo += static_cast<int64_t>(morder[k].size());
            obj_mask_off[k + 1] = mo;
            for (int32_t x : sets[k].t)
                if (x >= 0) obj_pts[po++] = x;
            obj_pt_off[k + 1] = po;
            son_off[k + 1] = comp_off[k + 1];
        }
        std::copy(comp_mem.begin(), comp_mem.end(), son_order);
        return MC_OK;
    } catch (const std::bad_alloc &) {
        return MC_ERR_HIP;
    }
}

extern "C" int mc_setorder_replay(int32_t num_levels, const int32_t *level_sizes, const int64_t *edge_off,
                                  const int32_t *edge_a, const int32_t *edge_b, const int64_t *pt_off,
                                  const int32_t *pts, int32_t num_threads, int32_t *num_objects,
                                  int64_t *obj_mask_off, int32_t *mask_order, int64_t *obj_pt_off, int32_t *obj_pts,
                                  int64_t *son_off, int32_t *son_order, int32_t *labels)
{
    if (num_levels < 1 || !level_sizes || !pt_off || level_sizes[0] < 0 || pt_off[0] != 0) return MC_ERR_INVALID;
    const int N0 = level_sizes[0];
    std::vector<int64_t> start(static_cast<size_t>(N0)), len(static_cast<size_t>(N0));
    for (int i = 0; i < N0; i++) {
        if (pt_off[i + 1] < pt_off[i]) return MC_ERR_INVALID;
        start[i] = pt_off[i];
        len[i] = pt_off[i + 1] - pt_off[i];
    }
    mc_setorder *h = nullptr;
    int rc = mc_setorder_begin(N0, start.data(), len.data(), pts, num_threads, 0, &h);
    if (rc != MC_OK) return rc;
    rc = mc_setorder_finish(h, num_levels, level_sizes, edge_off, edge_a, edge_b, num_objects, obj_mask_off, mask_order,
                            obj_pt_off, obj_pts, son_off, son_order, labels);
    mc_setorder_free(h);
    return rc;
}

// lachain_amd/csrc/lcb_queue.cpp — in-library aggregation queue for one-share-per-call callers.
//
// The reference verifies one share per call, from one thread per protocol instance:
//   HoneyBadger.HandleDecryptedMessage -> PublicKey.VerifyShare   (src/Lachain.Consensus/HoneyBadger/HoneyBadger.cs:211-212)
//   HoneyBadger.HandleCommonSubset filter                         (HoneyBadger.cs:156-158)
//   ThresholdSigner.AddShare -> IsShareValid -> ValidateSignature  (src/Lachain.Crypto/ThresholdSignature/ThresholdSigner.cs:62)
//   threads: AbstractProtocol.cs:46-47
// A GPU launch per share would be latency-bound, so callers submit single shares and get a ticket; worker threads flush
// the pending shares as ONE batch (lcb_tpke_verify_shares_cached / lcb_ts_verify_shares on the worker's own context)
// when max_batch shares are pending or the oldest pending share is max_delay_us old, and lcb_queue_wait(ticket)
// returns that share's decision.  Ciphertexts, verification keys and messages are de-duplicated per batch, so the batch
// shares hash-to-G2 and Miller-line precomputation exactly as a caller-built batch would.  Decisions are the
// same per-share results the batch entry points produce (bit-exact with VerifyShare / ValidateSignature).
// lcb_queue_set_batched(q, m) sends flushes of at least m shares through the randomized batch checks instead
// (k_batch.hip): more shares per GPU-second, a few more latency-bound launches per flush.
//
// Flushes overlap (round 5): a flush is a serial chain of latency-bound launches (decompression, the nine-lane Miller
// loop and final exponentiation: ~5 ms whatever its size) that leaves the GPU nearly idle, so three workers
// (LCB_QUEUE_WORKERS_DEFAULT), each with its own thread context and stream, take due shares from ONE pending list: a
// share waits for the deadline and a free worker, not for the flush in progress to end and then its own (round 4: two
// workers with ciphertext affinity, ~1.5 flushes per share).  Each worker's context keeps the prepared line sets of the
// ciphertexts it has seen and the decompressed verification keys, and lcb_queue_tpke_prepare(ct) prepares a ciphertext
// ahead of its shares — the reference decrypts every ciphertext of the common subset (PrivateKey.Decrypt, which hashes
// U || V to G2: HoneyBadger.cs:144-146) before the other validators' decryption shares for it are handled
// (HoneyBadger.cs:190-213), so no flush waits for hash-to-G2 and two line sets.  Round 6: the ciphertext is
// prepared at once by ONE worker (round robin), and by the others only while they have no due shares and no
// preparation of their own, so a stream of prepares never holds every worker away from due shares.  A share of a
// ciphertext its flushing worker has not prepared is prepared by that worker in the flush (and cached there).
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/lachain_bls.h"

namespace {
using clk = std::chrono::steady_clock;

struct TpkeItem {
    int64_t ticket;
    std::string key, ct;   // key = Y (48 B); ct = U (48) || W (96) || V
    uint8_t ui[48];
};
struct TsItem {
    int64_t ticket;
    std::string pk, msg;   // pk 48 B
    uint8_t sig[96];
};
}  // namespace

#define LCB_QUEUE_WORKERS 4      // most flushes in flight (LCB_QUEUE_WORKERS in the environment: 1 .. 4)
#define LCB_QUEUE_WORKERS_DEFAULT 3   // three: at the default GPU_MAX_HW_QUEUES = 4 a fourth worker's stream shares a
                                      // hardware queue with another's, and a flush queued behind a flush doubles its
                                      // latency (profiles/r05/queue/ab.txt: p90 10.6-10.9 ms at four, 6.7 at three)
#define LCB_QUEUE_PREP_CHUNK 1024  // ciphertexts per preparation call (the widest batch the context cache takes)
#define LCB_QUEUE_IDLE_CHUNK 64    // ciphertexts per idle-time preparation (one wave of the preparation kernel)
struct lcb_queue {
    std::mutex mu;
    std::condition_variable cv_work, cv_done;
    size_t max_batch;
    std::chrono::microseconds max_delay;
    std::vector<TpkeItem> tpke;                        // any worker
    clk::time_point oldest;
    std::vector<std::string> prep[LCB_QUEUE_WORKERS];  // ciphertexts this worker prepares before anything else
    std::vector<std::string> idle_prep[LCB_QUEUE_WORKERS];   // ... and the others' ones, when it has nothing due
    uint32_t prep_rr = 0;                              // round robin over the workers for the eager preparation
    std::vector<TsItem> ts;                            // any worker
    clk::time_point ts_oldest;
    bool stop = false, flush_now = false;
    int64_t next_ticket = 1;
    std::unordered_map<int64_t, int8_t> results;     // ticket -> 1 / 0 / -1 (batch failed), until waited for
    std::set<int64_t> open;                           // tickets submitted whose result is not yet produced
    uint64_t batches = 0, items = 0, max_seen = 0;
    // randomized batch checks (lcb_queue_set_batched): flushes of at least batched_min shares go through the
    // *_batched entry points, shares ordered by ciphertext / message so each one's shares form a group
    size_t batched_min = 0;
    std::string last_error;
    // the workers, each with its own thread context (prepared-ciphertext and key caches) and stream
    std::vector<std::thread> workers;
    int n_workers = LCB_QUEUE_WORKERS_DEFAULT;
    uint64_t prepared = 0;
};

namespace {

void run_tpke(lcb_queue *q, std::vector<TpkeItem> &items, size_t batched_min) {
    std::unordered_map<std::string, uint32_t> kidx, cidx;
    std::vector<uint8_t> keys, us, ws, vs, uis(48 * items.size());
    std::vector<uint32_t> voff(1, 0), ct(items.size()), dec(items.size());
    for (size_t i = 0; i < items.size(); i++) {
        TpkeItem &it = items[i];
        auto k = kidx.emplace(it.key, (uint32_t)kidx.size());
        if (k.second) keys.insert(keys.end(), it.key.begin(), it.key.end());
        auto c = cidx.emplace(it.ct, (uint32_t)cidx.size());
        if (c.second) {
            const uint8_t *b = (const uint8_t *)it.ct.data();
            us.insert(us.end(), b, b + 48);
            ws.insert(ws.end(), b + 48, b + 144);
            vs.insert(vs.end(), b + 144, b + it.ct.size());
            voff.push_back((uint32_t)vs.size());
        }
        dec[i] = k.first->second;
        ct[i] = c.first->second;
        memcpy(&uis[48 * i], it.ui, 48);
    }
    std::vector<uint8_t> acc(items.size());
    if (vs.empty()) vs.push_back(0);
    int rc;
    if (batched_min && items.size() >= batched_min) {
        // ciphertext-major order for the group checks (stable: a ciphertext's shares keep their submission order)
        std::vector<uint32_t> ord(items.size());
        for (size_t i = 0; i < ord.size(); i++) ord[i] = (uint32_t)i;
        std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return ct[a] < ct[b]; });
        std::vector<uint32_t> ct2(ord.size()), dec2(ord.size());
        std::vector<uint8_t> uis2(uis.size()), acc2(ord.size());
        for (size_t j = 0; j < ord.size(); j++) {
            ct2[j] = ct[ord[j]];
            dec2[j] = dec[ord[j]];
            memcpy(&uis2[48 * j], &uis[48 * (size_t)ord[j]], 48);
        }
        rc = lcb_tpke_verify_shares_batched(acc2.data(), items.size(), keys.data(), kidx.size(), us.data(), ws.data(),
                                            vs.data(), voff.data(), cidx.size(), ct2.data(), dec2.data(), uis2.data());
        for (size_t j = 0; j < ord.size(); j++) acc[ord[j]] = acc2[j];
    } else {
        // the worker thread's context keeps a ciphertext's prepared line sets across flushes (its N shares arrive over
        // several of them)
        rc = lcb_tpke_verify_shares_cached(acc.data(), items.size(), keys.data(), kidx.size(), us.data(), ws.data(),
                                           vs.data(), voff.data(), cidx.size(), ct.data(), dec.data(), uis.data());
    }
    std::lock_guard<std::mutex> lk(q->mu);
    if (rc) q->last_error = lcb_last_error();
    for (size_t i = 0; i < items.size(); i++) {
        q->results[items[i].ticket] = rc ? -1 : (int8_t)(acc[i] != 0);
        q->open.erase(items[i].ticket);
    }
}

void run_ts(lcb_queue *q, std::vector<TsItem> &items, size_t batched_min) {
    std::unordered_map<std::string, uint32_t> pidx, midx;
    std::vector<uint8_t> pks, msgs, sigs(96 * items.size());
    std::vector<uint32_t> moff(1, 0), mi(items.size()), pi(items.size());
    for (size_t i = 0; i < items.size(); i++) {
        TsItem &it = items[i];
        auto p = pidx.emplace(it.pk, (uint32_t)pidx.size());
        if (p.second) pks.insert(pks.end(), it.pk.begin(), it.pk.end());
        auto m = midx.emplace(it.msg, (uint32_t)midx.size());
        if (m.second) {
            msgs.insert(msgs.end(), it.msg.begin(), it.msg.end());
            moff.push_back((uint32_t)msgs.size());
        }
        pi[i] = p.first->second;
        mi[i] = m.first->second;
        memcpy(&sigs[96 * i], it.sig, 96);
    }
    std::vector<uint8_t> acc(items.size());
    if (msgs.empty()) msgs.push_back(0);
    int rc;
    if (batched_min && items.size() >= batched_min) {
        std::vector<uint32_t> ord(items.size());
        for (size_t i = 0; i < ord.size(); i++) ord[i] = (uint32_t)i;
        std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return mi[a] < mi[b]; });
        std::vector<uint32_t> mi2(ord.size()), pi2(ord.size());
        std::vector<uint8_t> sigs2(sigs.size()), acc2(ord.size());
        for (size_t j = 0; j < ord.size(); j++) {
            mi2[j] = mi[ord[j]];
            pi2[j] = pi[ord[j]];
            memcpy(&sigs2[96 * j], &sigs[96 * (size_t)ord[j]], 96);
        }
        rc = lcb_ts_verify_shares_batched(acc2.data(), items.size(), pks.data(), pidx.size(), sigs2.data(), msgs.data(),
                                          moff.data(), midx.size(), mi2.data(), pi2.data());
        for (size_t j = 0; j < ord.size(); j++) acc[ord[j]] = acc2[j];
    } else {
        rc = lcb_ts_verify_shares(acc.data(), items.size(), pks.data(), pidx.size(), sigs.data(), msgs.data(),
                                  moff.data(), midx.size(), mi.data(), pi.data());
    }
    std::lock_guard<std::mutex> lk(q->mu);
    if (rc) q->last_error = lcb_last_error();
    for (size_t i = 0; i < items.size(); i++) {
        q->results[items[i].ticket] = rc ? -1 : (int8_t)(acc[i] != 0);
        q->open.erase(items[i].ticket);
    }
}

// prepare ciphertexts (U || W || V) into this worker's cache: the cached verify with no shares
void run_prepare(lcb_queue *q, std::vector<std::string> &cts) {
    std::unordered_map<std::string, uint32_t> cidx;
    std::vector<uint8_t> us, ws, vs;
    std::vector<uint32_t> voff(1, 0);
    for (auto &ct : cts) {
        if (!cidx.emplace(ct, (uint32_t)cidx.size()).second) continue;
        const uint8_t *b = (const uint8_t *)ct.data();
        us.insert(us.end(), b, b + 48);
        ws.insert(ws.end(), b + 48, b + 144);
        vs.insert(vs.end(), b + 144, b + ct.size());
        voff.push_back((uint32_t)vs.size());
    }
    if (vs.empty()) vs.push_back(0);
    int rc = 0;
    for (size_t k0 = 0; k0 < cidx.size() && !rc; k0 += LCB_QUEUE_PREP_CHUNK) {
        const size_t m = std::min((size_t)LCB_QUEUE_PREP_CHUNK, cidx.size() - k0);
        std::vector<uint32_t> vo(voff.begin() + k0, voff.begin() + k0 + m + 1);
        rc = lcb_tpke_verify_shares_cached(nullptr, 0, nullptr, 0, us.data() + 48 * k0, ws.data() + 96 * k0, vs.data(),
                                           vo.data(), m, nullptr, nullptr, nullptr);
    }
    std::lock_guard<std::mutex> lk(q->mu);
    if (rc) q->last_error = lcb_last_error();
    else q->prepared += cidx.size();
}

void worker_loop(lcb_queue *q, int w) {
    std::unique_lock<std::mutex> lk(q->mu);
    for (;;) {
        const size_t pt = q->tpke.size(), ps = q->ts.size(), pp = q->prep[w].size(), pi = q->idle_prep[w].size();
        if (pt + ps + pp + pi == 0) {
            if (q->stop) return;
            q->cv_work.wait(lk);
            continue;
        }
        const clk::time_point now = clk::now();
        const bool due_t = pt && (q->stop || q->flush_now || pt >= q->max_batch || now >= q->oldest + q->max_delay);
        const bool due_s = ps && (q->stop || q->flush_now || ps >= q->max_batch || now >= q->ts_oldest + q->max_delay);
        if (!pp && !due_t && !due_s && !pi) {
            clk::time_point next = clk::time_point::max();
            if (pt) next = std::min(next, q->oldest + q->max_delay);
            if (ps) next = std::min(next, q->ts_oldest + q->max_delay);
            q->cv_work.wait_until(lk, next);
            continue;
        }
        std::vector<TpkeItem> t;
        std::vector<TsItem> s;
        std::vector<std::string> p;
        p.swap(q->prep[w]);
        if (p.empty()) {              // this worker's preparations first: the shares it takes then hit its cache
            if (due_t) t.swap(q->tpke);
            if (due_s) s.swap(q->ts);
            if (t.empty() && s.empty() && pi) {      // nothing due: prepare the others' ciphertexts here too, in
                auto &ip = q->idle_prep[w];          // chunks, so due shares find this worker free again soon
                const size_t m = std::min(ip.size(), (size_t)LCB_QUEUE_IDLE_CHUNK);
                p.assign(std::make_move_iterator(ip.begin()), std::make_move_iterator(ip.begin() + (long)m));
                ip.erase(ip.begin(), ip.begin() + (long)m);
            }
        }
        if (q->tpke.empty() && q->ts.empty()) q->flush_now = false;
        const size_t batched_min = q->batched_min;     // read under the lock (lcb_queue_set_batched writes it)
        const size_t pending = t.size() + s.size();
        if (pending) {
            q->batches++;
            q->items += pending;
            if (pending > q->max_seen) q->max_seen = pending;
        }
        lk.unlock();
        if (!p.empty()) run_prepare(q, p);
        if (!t.empty()) run_tpke(q, t, batched_min);
        if (!s.empty()) run_ts(q, s, batched_min);
        lk.lock();
        if (pending) q->cv_done.notify_all();
        else q->cv_work.notify_all();   // due shares this worker left while it prepared: another worker may be idle
    }
}

void wake(lcb_queue *q, size_t pending, size_t max_batch) {
    if (pending == 1 || pending >= max_batch) q->cv_work.notify_all();
}

}  // namespace

extern "C" lcb_queue *lcb_queue_create(size_t max_batch, uint32_t max_delay_us) {
    lcb_queue *q = new lcb_queue;
    q->max_batch = max_batch ? max_batch : 1;
    q->max_delay = std::chrono::microseconds(max_delay_us);
    if (const char *e = getenv("LCB_QUEUE_WORKERS")) {    // A/B knob: 1 .. LCB_QUEUE_WORKERS
        const int k = atoi(e);
        if (k >= 1 && k <= LCB_QUEUE_WORKERS) q->n_workers = k;
    }
    for (int k = 0; k < q->n_workers; k++) q->workers.emplace_back(worker_loop, q, k);
    return q;
}
extern "C" void lcb_queue_destroy(lcb_queue *q) {
    if (!q) return;
    {
        std::lock_guard<std::mutex> lk(q->mu);
        q->stop = true;
    }
    q->cv_work.notify_all();
    for (auto &w : q->workers) w.join();
    q->cv_done.notify_all();
    delete q;
}
extern "C" int64_t lcb_queue_tpke_verify(lcb_queue *q, const uint8_t y48[48], const uint8_t u48[48], const uint8_t *v,
                                         size_t v_len, const uint8_t w96[96], const uint8_t ui48[48]) {
    if (!q || !y48 || !u48 || !w96 || !ui48 || (v_len && !v)) return -1;
    TpkeItem it;
    it.key.assign((const char *)y48, 48);
    it.ct.reserve(144 + v_len);
    it.ct.append((const char *)u48, 48);
    it.ct.append((const char *)w96, 96);
    if (v_len) it.ct.append((const char *)v, v_len);
    memcpy(it.ui, ui48, 48);
    std::unique_lock<std::mutex> lk(q->mu);
    if (q->stop) return -1;
    it.ticket = q->next_ticket++;
    q->open.insert(it.ticket);
    q->tpke.push_back(std::move(it));
    const size_t pending = q->tpke.size();
    if (pending == 1) q->oldest = clk::now();
    wake(q, pending, q->max_batch);
    return q->next_ticket - 1;
}
extern "C" int lcb_queue_tpke_prepare(lcb_queue *q, const uint8_t u48[48], const uint8_t *v, size_t v_len,
                                      const uint8_t w96[96]) {
    if (!q || !u48 || !w96 || (v_len && !v)) return -1;
    std::string ct;
    ct.reserve(144 + v_len);
    ct.append((const char *)u48, 48);
    ct.append((const char *)w96, 96);
    if (v_len) ct.append((const char *)v, v_len);
    std::lock_guard<std::mutex> lk(q->mu);
    if (q->stop) return -1;
    const int owner = (int)(q->prep_rr++ % (uint32_t)q->n_workers);
    for (int w = 0; w < q->n_workers; w++) (w == owner ? q->prep[w] : q->idle_prep[w]).push_back(ct);
    q->cv_work.notify_all();
    return 0;
}
extern "C" int64_t lcb_queue_ts_verify(lcb_queue *q, const uint8_t pk48[48], const uint8_t *msg, size_t msg_len,
                                       const uint8_t sig96[96]) {
    if (!q || !pk48 || !sig96 || (msg_len && !msg)) return -1;
    TsItem it;
    it.pk.assign((const char *)pk48, 48);
    if (msg_len) it.msg.assign((const char *)msg, msg_len);
    memcpy(it.sig, sig96, 96);
    std::unique_lock<std::mutex> lk(q->mu);
    if (q->stop) return -1;
    it.ticket = q->next_ticket++;
    q->open.insert(it.ticket);
    q->ts.push_back(std::move(it));
    const size_t pending = q->ts.size();
    if (pending == 1) q->ts_oldest = clk::now();
    wake(q, pending, q->max_batch);
    return q->next_ticket - 1;
}
extern "C" int lcb_queue_flush(lcb_queue *q) {
    if (!q) return -1;
    {
        std::lock_guard<std::mutex> lk(q->mu);
        q->flush_now = true;
    }
    q->cv_work.notify_all();
    return 0;
}
extern "C" int lcb_queue_wait(lcb_queue *q, int64_t ticket) {
    if (!q || ticket <= 0) return -1;
    std::unique_lock<std::mutex> lk(q->mu);
    if (ticket >= q->next_ticket) return -1;
    for (;;) {
        auto it = q->results.find(ticket);
        if (it != q->results.end()) {
            int r = it->second;
            q->results.erase(it);
            return r;
        }
        if (!q->open.count(ticket)) return -1;   // already waited for
        q->cv_done.wait(lk);
    }
}
extern "C" const char *lcb_queue_last_error(lcb_queue *q) { return q ? q->last_error.c_str() : ""; }
extern "C" int lcb_queue_set_batched(lcb_queue *q, size_t min_shares) {
    if (!q) return -1;
    std::lock_guard<std::mutex> lk(q->mu);
    q->batched_min = min_shares;
    return 0;
}
extern "C" int lcb_queue_stats(lcb_queue *q, uint64_t out[3]) {
    if (!q || !out) return -1;
    std::lock_guard<std::mutex> lk(q->mu);
    out[0] = q->batches;
    out[1] = q->items;
    out[2] = q->max_seen;
    return 0;
}

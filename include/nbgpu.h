/*
 * nbgpu.h — C-ABI of the MI355X-native Maglev flow-steering path.
 *
 * This is the drop-in boundary for NetBricks' test/maglev hot path.  The
 * reference runs, per packet, inside its batch operators:
 *
 *   parse::<MacHeader>()            framework/src/operators/mod.rs:59-64
 *   transform(swap_addresses)       test/maglev/src/nf.rs:94-98, headers/mac.rs:140-145
 *   group_by(ct, group_fn)          test/maglev/src/nf.rs:99-108, operators/group_by.rs:43-55
 *     group_fn = lut[fnv(flow) % M] test/maglev/src/nf.rs:101-106, utils/flow.rs:53-62,96-110
 *
 * A per-packet FFI call is infeasible, so the boundary sits at the batch level:
 * one call classifies a whole batch (parse + MAC swap + 5-tuple FNV-1a + Maglev
 * lookup) and emits the per-group FIFO order that the reference's MPSC queues
 * hold (framework/src/queues/mpsc_mbuf_queue.rs:91-115,197-212).  Plain C types
 * only; device pointers are caller-owned HBM allocations.
 *
 * Errors: 0 on success, negative errno-style codes otherwise, mirroring
 * libzcsi (native/pmd.c:128,154,165; native/init.c:176-177).  The message of
 * the last error on the calling thread is returned by nbg_last_error().
 *
 * Threading: a handle is used by one thread / one stream at a time (the
 * reference runs one pipeline per pinned scheduler core, scheduler/context.rs:55-69).
 * Use one handle per concurrent stream.  A handle remembers the stream of its
 * last call: a later call on another stream is ordered after the work issued
 * there (an event recorded on it), and nbg_maglev_check synchronises it.  So
 * the stream a call names must stay valid until the handle's next call
 * returns, or until nbg_maglev_destroy (destroy a per-burst stream only after
 * that).
 */
#ifndef NBGPU_H
#define NBGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NBG_OK 0
#define NBG_EINVAL (-22)
#define NBG_ENOMEM (-12)
#define NBG_ENODEV (-19)
#define NBG_EIO (-5)
#define NBG_EBUSY (-16)
#define NBG_ETIMEDOUT (-110)

/* backend value for a packet on which the reference would panic:
 * data_len < 14 (Packet::parse_header assert, interface/packet.rs:392-399) or a
 * payload shorter than max(20, 4*IHL+4) (slice OOB in utils/flow.rs:53-62).
 * Such packets land in group n_backends (the last of n_backends+1 groups). */
#define NBG_SENTINEL 0xFFFFu

/*
 * Recommended path per configuration (BASELINE.json configs; DESIGN.md has the measurements):
 *   C1  host mbufs, 10k-packet pcap      nbg_maglev_host_submit / _wait (or nbg_host_register + zero copy)
 *   C2  1M fixed 64-B slots, 65 backends several RX queues resident: nbg_maglev_classify_device_multi;
 *                                         a stream of batches: the persistent ring (nbg_ring_*) with
 *                                         nbg_ring_group_burst; one batch: nbg_maglev_classify_device
 *   C3  IMIX descriptors, 1000 backends  several RX queues: nbg_maglev_classify_desc_multi (up to 16 batches
 *                                         per launch); one batch: nbg_maglev_classify_device; NBG_OWNED_WINDOWS
 *   C4  C2 in 8 shards, one per GPU      per rank: the persistent ring + nbg_ring_group_burst
 *   C5  lpm -> maglev, IMIX              several RX queues: nbg_chain_lpm_maglev_multi; one batch:
 *                                         nbg_chain_lpm_maglev_device; NBG_OWNED_WINDOWS
 */

/* classify flags */
#define NBG_SWAP_MACS 0x1u      /* apply MacHeader::swap_addresses in place (nf.rs:94-98) */
#define NBG_OWNED_WINDOWS 0x4u  /* descriptor mode: the 64 B at every packet start belong to that
                                   packet (true for DPDK mbufs, whose data room is >= 2 KiB) */
#define NBG_WB_PARTIAL 0x8u     /* write back only the 16 B holding the MACs: the zero-copy host path
                                   (nbg_host_register), where the rewrite crosses PCIe */
#define NBG_DEFER_GROUP 0x10u   /* launch only the classify kernel; nbg_maglev_finish_group launches
                                   the grouping kernel (e.g. on another stream, after an event) */

/* Measured variants: not the recommended paths (each measured slower than the default on the
 * bench's workloads, DESIGN.md "Measured variants"), kept as named A/B alternatives and covered by
 * the parity fuzz.  NBG_LUT_TILED is BASELINE config C3's named "LDS-tiled table". */
#define NBG_LUT_LDS 0x2u        /* stage the LUT in LDS per workgroup instead of gathering from L2
                                   (u8/u16 LUT <= 72 KiB; lower occupancy) */
#define NBG_LUT_TILED 0x20u     /* u16 LUTs (> 256 backends): instead of gathering from L2, bucket the
                                   packets by 64-KiB LUT tile and look them up per tile in LDS */
#define NBG_STREAM_DESC 0x40u   /* descriptor layouts with NBG_OWNED_WINDOWS, >= 262144 packets: the
                                   streaming classify kernel (one block per CU, everything fetched by
                                   LDS-DMA).  Faster on one stream, slower when several streams share
                                   the GPU (it cannot co-run) */
#define NBG_GROUP_LAG 0x80u     /* pipelined grouping for a producer that calls the handle back to back
                                   (GroupByProducer::execute, operators/group_by.rs:43-55): the call
                                   classifies its batch (backend[], MAC swap) and leaves the batch's
                                   grouping pending; the handle's next classify call groups it inside
                                   its own classify launch (or launches it first, when that call cannot
                                   carry it), and nbg_maglev_finish_group launches it alone.  So
                                   d_perm / d_counts of call i are complete once the work of call i+1
                                   (or of finish_group) is, in stream order; the call's buffers must
                                   stay untouched until then.  Carried for fixed 64-B-aligned slots,
                                   >= 262144 packets, <= 255 backends, M <= 65537 and partitions x bins
                                   within the direct-scan limit; other batches are grouped at once.
                                   Not with NBG_DEFER_GROUP or in a graph capture. */

typedef struct nbg_maglev nbg_maglev;

/* Build the Maglev LUT on the host exactly as Maglev::new (nf.rs:70-76:
 * offset_skip_for_name nf.rs:21-31, generate_lut nf.rs:44-68) and upload it to
 * `device`.  names[i] has name_lens[i] bytes (UTF-8, no terminator needed).
 * Replaces: `Maglev::new(backends, 65537)` at test/maglev/src/nf.rs:90.
 * table_size must be >= 2 (the reference hard-codes 65537); n_backends in [1, 65534]. */
int nbg_maglev_create(const char* const* names, const uint32_t* name_lens, uint32_t n_backends,
                      uint64_t table_size, int device, nbg_maglev** out);

/* Same as nbg_maglev_create but adopts a LUT the caller already holds (e.g. one
 * broadcast over RCCL from rank 0): lut[j] < n_backends for all j. */
int nbg_maglev_create_from_lut(const uint16_t* lut, uint64_t table_size, uint32_t n_backends, int device,
                               nbg_maglev** out);

void nbg_maglev_destroy(nbg_maglev* h);

uint32_t nbg_maglev_backends(const nbg_maglev* h);
uint64_t nbg_maglev_table_size(const nbg_maglev* h);

/* Copy the LUT (entries as u16; the reference stores usize) to host memory `out` of n entries. */
int nbg_maglev_lut(const nbg_maglev* h, uint16_t* out, uint64_t n);

/* Pre-allocate the per-call scratch for batches of up to max_pkts packets so that
 * later classify calls allocate nothing (needed before hipGraph capture). */
int nbg_maglev_reserve(nbg_maglev* h, uint64_t max_pkts);

/*
 * Device-resident batch classify (the hot path).  Replaces the per-packet loop of
 * GroupByProducer::execute (operators/group_by.rs:43-55) for a whole batch.
 *
 *   d_pkts     packet bytes in HBM; packet i starts at d_pkts + (d_off ? d_off[i] : i*stride)
 *   d_off      nullable u32 byte offsets (descriptor mode, e.g. IMIX)
 *   d_len      nullable u16 frame lengths (mbuf data_len); NULL => every frame is fixed_len
 *   n_pkts     packets in the batch, < 2^30
 *   flags      NBG_SWAP_MACS | NBG_LUT_LDS | NBG_OWNED_WINDOWS | NBG_DEFER_GROUP | NBG_LUT_TILED |
 *              NBG_STREAM_DESC | NBG_GROUP_LAG
 *   d_backend  out, n_pkts u16: backend index, or NBG_SENTINEL
 *   d_perm     out (nullable), n_pkts u32: packet indices grouped by backend 0..n-1 then the
 *              sentinel group, ascending index inside each group (per-group FIFO order)
 *   d_counts   out (nullable unless d_perm set), n_backends+1 u32: group sizes
 *   stream     hipStream_t (NULL = default stream); the call is asynchronous
 *
 * Frames shorter than 48 B, unaligned or with IHL != 5 take a byte-wise slow path
 * with identical results.  The kernel reads (and, with NBG_SWAP_MACS, rewrites with
 * their own values) the bytes of the 64-B window at each packet start that lie inside
 * the frame, or the whole window when it is owned: fixed slots with stride >= 64, or
 * NBG_OWNED_WINDOWS.  Windows of distinct packets must not overlap in that case.
 */
int nbg_maglev_classify_device(nbg_maglev* h, uint8_t* d_pkts, const uint32_t* d_off, const uint16_t* d_len,
                               uint32_t stride, uint16_t fixed_len, uint64_t n_pkts, uint32_t flags,
                               uint16_t* d_backend, uint32_t* d_perm, uint32_t* d_counts, void* stream);

/* As nbg_maglev_classify_device, plus d_mac_out (nullable, n_pkts x 12 B): with NBG_SWAP_MACS
 * the swapped MAC pair of packet i (its new bytes 0..11) is written to d_mac_out + 12*i and
 * the packet bytes are left untouched — the egress rewrite record a host-mbuf pipeline
 * applies before TX.  Packets shorter than 14 B get no record (their 12 bytes are left as they
 * were). */
int nbg_maglev_classify_device_ex(nbg_maglev* h, uint8_t* d_pkts, const uint32_t* d_off, const uint16_t* d_len,
                                  uint32_t stride, uint16_t fixed_len, uint64_t n_pkts, uint32_t flags,
                                  uint16_t* d_backend, uint32_t* d_perm, uint32_t* d_counts, uint8_t* d_mac_out,
                                  void* stream);

/*
 * Several device-resident batches in one launch of each kernel: what NetBricks does with the
 * batches of several RX queues, one pipeline each (scheduler/context.rs:241-255), when they are
 * classified together.  Every batch keeps its own outputs, exactly as if it were passed alone to
 * nbg_maglev_classify_device_ex with the same stride / fixed_len / flags: backend[], the MAC swap
 * (in place, or records in d_mac_out), and its own perm / counts (grouped per batch, never across
 * batches).  Fused (one streaming-classify launch + one group launch over all batches) for fixed
 * 64-B-aligned slots (stride % 16 == 0, stride >= 64, fixed_len >= 48, 16-B aligned d_pkts), at
 * most 255 backends, M <= 65537 and at least 262144 packets in all; otherwise the batches are run
 * one after another through nbg_maglev_classify_device_ex on `stream`.  1 <= n_batches <=
 * NBG_MAX_MULTI.  Flags: NBG_SWAP_MACS, and NBG_DEFER_GROUP on the fused path (nbg_maglev_finish_group
 * then launches the one group kernel of all batches); others are NBG_EINVAL.  While a persistent ring
 * runs on the device the fused path (a streaming kernel) is not taken, so NBG_DEFER_GROUP is then
 * NBG_EINVAL too; a ring stops holding the device once its kernel has ended (stop or idle exit).
 * Either every batch has d_perm (or d_counts) or none has.
 */
#define NBG_MAX_MULTI 16u
typedef struct nbg_batch {
  uint8_t* d_pkts;
  uint64_t n_pkts;
  uint16_t* d_backend;
  uint32_t* d_perm;    /* nullable */
  uint32_t* d_counts;  /* nullable unless d_perm set (then n_backends + 1 u32) */
  uint8_t* d_mac_out;  /* nullable: 12-B swapped-MAC records instead of the in-place swap */
} nbg_batch;
int nbg_maglev_classify_device_multi(nbg_maglev* h, const nbg_batch* batches, uint32_t n_batches, uint32_t stride,
                                     uint16_t fixed_len, uint32_t flags, void* stream);

/*
 * The same for descriptor batches (IMIX: a u32 byte offset and a u16 frame length per packet, the
 * layout of configs C3 and C5): one tile-per-wave classify launch over all batches, then (grouping)
 * one hist, one scan and one group launch over all of them.  Each batch's outputs are exactly those
 * of nbg_maglev_classify_device (or nbg_chain_lpm_maglev_device, with d_gate) on that batch alone
 * with the same flags.  One launch pays the classify kernel's ramp and tail (~6.7 us, a quarter of
 * a 1M IMIX batch) once for all batches (DESIGN.md sections 4 and 6).
 * Flags: NBG_SWAP_MACS (ignored by the chain: the two swaps cancel), NBG_OWNED_WINDOWS,
 * NBG_DEFER_GROUP (nbg_maglev_finish_group launches the grouping of all batches); others are
 * NBG_EINVAL.  d_off, d_len and d_backend (and d_gate for the chain) are required for a non-empty
 * batch.  More than 1023 backends with grouping: the batches run one after another.
 */
typedef struct nbg_desc_batch {
  uint8_t* d_pkts;
  const uint32_t* d_off;
  const uint16_t* d_len;
  uint64_t n_pkts;
  uint16_t* d_backend;
  uint32_t* d_perm;    /* nullable */
  uint32_t* d_counts;  /* nullable unless d_perm set (then n_backends + 1 u32) */
  uint16_t* d_gate;    /* the chain's lpm gate per packet; unused by nbg_maglev_classify_desc_multi */
} nbg_desc_batch;
int nbg_maglev_classify_desc_multi(nbg_maglev* h, const nbg_desc_batch* batches, uint32_t n_batches, uint32_t flags,
                                   void* stream);

/*
 * Persistent RX ring (the GPUDirect RX model: an RX queue that never stops, ReceiveBatch::execute
 * polling its port, framework/src/operators/receive_batch.rs:26,52-61).  nbg_ring_start launches ONE
 * streaming-classify kernel on `stream` (one block per CU: CUs - 1 classify blocks and a relay
 * block) that runs until nbg_ring_stop: it stages the LUT in LDS once and classifies batches as
 * they are posted, so no launch, LUT staging or pipeline ramp is paid per batch.  nbg_ring_post
 * hands it one device-resident batch of fixed slots (the streaming kernel's layout: stride % 16 ==
 * 0, 64 <= stride < 2^24, fixed_len >= 48, d_pkts and d_backend 16-B aligned) through a descriptor
 * ring in pinned host memory (the relay block copies it into HBM; no classify CU reads host
 * memory), and returns its ticket (0, 1, 2, ... in post order) without waiting; a post finds a free
 * slot first (NBG_RING_SLOTS batches may be outstanding).  nbg_ring_post_burst posts the first
 * batches of an array (an RX burst) without waiting: as many as there are free slots, reported in
 * *n_posted, the first one's ticket in *first_ticket.  Batch `ticket` is complete when nbg_ring_poll
 * reports more than `ticket` completed batches, or nbg_ring_wait(ticket) returns: its backend[] and
 * (NBG_SWAP_MACS) its in-place MAC swap are then in HBM, written through the L2, for any later
 * launch or copy.  Per packet the results are those of nbg_maglev_classify_device_ex with the same
 * arguments and no grouping (perm / counts are not produced on the ring).  Everything a post names
 * stays untouched by the caller until the batch is complete — including by a later post: a buffer is
 * posted again only once its previous batch is complete (the ring runs up to NBG_RING_SLOTS batches
 * at once, so two posts of one buffer could be classified concurrently).
 * The kernel runs on a private stream of the highest priority (a hardware queue no ordinary stream
 * shares: work queued behind a resident kernel would wait for it) and starts after the work issued
 * on `stream` so far.  It holds the LDS of every CU it occupies until it ends: after
 * nbg_ring_stop, or by itself after idle_ms without a post (its exit condition when the producer
 * goes away; 0 = 2000 ms; the next ring call then returns NBG_ETIMEDOUT).  nbg_ring_stop completes
 * every posted batch, waits for the kernel to end and for calls still blocked on the ring (other
 * producer threads' posts and waits, which then return) to leave, and keeps the ring's buffers for
 * the handle's next start: the ring pointer stays valid until nbg_maglev_destroy, and calls on a
 * stopped ring report its end.  NBG_EBUSY if the kernel did not end within idle_ms + 5 s: then
 * nothing it may touch is freed, the device stays busy, and every later call on the ring returns
 * NBG_EBUSY.
 * ONE ring per GPU: a second nbg_ring_start on a device whose ring runs (from any handle) returns
 * NBG_EBUSY at once.  Several RX queues share the device's ring through nbg_ring_queue_* below.
 * While a handle's ring runs, that handle's classify calls (device, multi, host, chain) return
 * NBG_EBUSY: their kernels would queue behind the resident one.  Other handles' batches on the same
 * device co-run in the LDS the ring leaves free (about 30 KB per CU in place): while a
 * ring runs they take the tile-per-wave classify kernel (never the streaming ones or NBG_LUT_LDS,
 * which need a whole CU's LDS), with identical results.  A grouping launch whose block would need
 * more LDS than that (many backends: the 1001-bin group block of C3 takes about 40 KB) takes the
 * compact group kernel while a ring runs (28 KB at 1001 bins), with identical results.
 * Requires <= 255 backends and M <= 65537 (the u8 LUT in LDS).
 * flags: 0 (read only) or NBG_SWAP_MACS (in place).
 * The nbg_ring_* calls of one ring are thread-safe (one mutex per ring).
 */
#define NBG_RING_SLOTS 64u
typedef struct nbg_ring nbg_ring;
int nbg_ring_start(nbg_maglev* h, uint32_t stride, uint16_t fixed_len, uint32_t flags, uint32_t idle_ms,
                   void* stream, nbg_ring** out);
int nbg_ring_post(nbg_ring* r, uint8_t* d_pkts, uint64_t n_pkts, uint16_t* d_backend, uint64_t* ticket);
typedef struct nbg_ring_batch {
  uint8_t* d_pkts;
  uint64_t n_pkts;
  uint16_t* d_backend;
} nbg_ring_batch;
int nbg_ring_post_burst(nbg_ring* r, const nbg_ring_batch* batches, uint32_t n_batches, uint32_t* n_posted,
                        uint64_t* first_ticket);
/* Group a ring batch: perm (u32[n], packet indices grouped by backend, arrival order inside a group)
 * and counts (u32[nb+1]) from its backend[], as nbg_maglev_classify_device_ex would give them
 * (group_by.rs:46-51).  Launches on `stream` (any caller stream) that co-run with the resident ring
 * kernel.  `ticket` must be among the last NBG_RING_SLOTS posted; it need not be complete yet: a
 * one-wave gate kernel ahead of the grouping waits on the stream for the ring's completion word in
 * HBM, so a producer enqueues a batch's grouping right after posting it, without polling (the
 * reference classifies and enqueues in one loop, operators/group_by.rs:43-55).  If the ring ends
 * before completing the batch (stop, idle exit), the gate opens anyway and perm / counts group
 * whatever backend[] holds (always inside perm's n entries); the ring's next call reports the end.
 * The batch's backend[] must stay untouched until the grouping has run on `stream`.
 * Up to 4 side streams group concurrently (one scratch set each; calls on one stream run in its
 * order); a further stream takes over the least recently used set after that set's stream's work. */
int nbg_ring_group(nbg_ring* r, uint64_t ticket, uint32_t* d_perm, uint32_t* d_counts, void* stream);
/* The same for the n_batches (1..NBG_MAX_MULTI) consecutive tickets first_ticket.. of an RX burst, with
 * one gate, one hist and one group launch for all of them (d_perm[j] / d_counts[j]: batch j's outputs):
 * a burst of shard-size batches costs the producer three launches instead of three per batch. */
int nbg_ring_group_burst(nbg_ring* r, uint64_t first_ticket, uint32_t n_batches, uint32_t* const* d_perm,
                         uint32_t* const* d_counts, void* stream);
int nbg_ring_poll(nbg_ring* r, uint64_t* completed);
int nbg_ring_wait(nbg_ring* r, uint64_t ticket, uint32_t timeout_ms);
int nbg_ring_stop(nbg_ring* r);

/*
 * RX queues on the device's ring: NetBricks runs one pipeline per RSS queue, each on its own core
 * (scheduler/context.rs:241-255; RSS in native/pmd.c:16).  Each queue's producer thread posts its
 * own batches into the one resident ring kernel and sees its own tickets (0, 1, 2, ... per queue),
 * its own completion count and its own grouping; the batches of all queues share the ring's
 * NBG_RING_SLOTS slots in the order they were posted.  Up to NBG_RING_MAX_QUEUES per ring; a queue
 * is used by one thread at a time (different queues from different threads).  nbg_ring_stop closes
 * every queue of the ring: later calls on a closed queue return NBG_EINVAL (a wait already blocked
 * when the ring stopped returns its batch's completion), and nbg_ring_queue_close frees it; queues
 * never closed are freed by nbg_maglev_destroy.  nbg_ring_queue_close before the stop closes and
 * frees one at once.
 */
#define NBG_RING_MAX_QUEUES 16u
typedef struct nbg_ring_queue nbg_ring_queue;
int nbg_ring_queue_open(nbg_ring* r, nbg_ring_queue** out);
int nbg_ring_queue_post(nbg_ring_queue* q, uint8_t* d_pkts, uint64_t n_pkts, uint16_t* d_backend, uint64_t* ticket);
int nbg_ring_queue_poll(nbg_ring_queue* q, uint64_t* completed);
int nbg_ring_queue_wait(nbg_ring_queue* q, uint64_t ticket, uint32_t timeout_ms);
int nbg_ring_queue_group(nbg_ring_queue* q, uint64_t ticket, uint32_t* d_perm, uint32_t* d_counts, void* stream);
int nbg_ring_queue_close(nbg_ring_queue* q);
/* The duration of the handle's last ring kernel (HIP events on its stream: start to end), valid after
 * nbg_ring_stop.  A stopped ring's buffers and stream are kept by the handle for its next
 * nbg_ring_start (freed by nbg_maglev_destroy). */
int nbg_ring_kernel_ms(nbg_maglev* h, float* ms);

/* Launch the grouping kernel of the last classify call made with NBG_DEFER_GROUP (or the pending
 * group of the last NBG_GROUP_LAG call) on `stream`; a stream other than the handle's last one is
 * ordered after it.  No-op when nothing is pending. */
int nbg_maglev_finish_group(nbg_maglev* h, void* stream);

/* Synchronise the handle's last stream and report any HIP error.  Not needed on the hot path. */
int nbg_maglev_check(nbg_maglev* h);

/*
 * Host-resident batch (the PCIe path): packet i is the mbuf data at pkt_ptrs[i]
 * with lens[i] bytes (MBuf::data_address / data_len, native/zcsi/mbuf.rs:34-49).
 * Header windows are gathered into pinned staging (with NBG_SWAP_MACS the MACs of every
 * frame of >= 14 B are swapped in the mbuf as its line is gathered: the flow hash reads
 * none of those 12 bytes), classified on the GPU, and the results copied back.
 * perm_out / counts_out are nullable.  Synchronous.  Replaces one GroupByProducer::execute
 * over a batch of host mbufs.
 */
int nbg_maglev_classify_host(nbg_maglev* h, uint8_t* const* pkt_ptrs, const uint16_t* lens, uint64_t n,
                             uint32_t flags, uint16_t* backend_out, uint32_t* perm_out, uint32_t* counts_out);

/*
 * The same, pipelined: nbg_maglev_host_submit gathers the batch's header windows into one of the
 * handle's NBG_HOST_SLOTS pinned staging slots (host worker threads; the MAC swap is applied to
 * the mbufs on the way), queues the H2D copy, the kernels and the D2H copy, and returns a ticket
 * without waiting; nbg_maglev_host_wait(ticket) waits for that batch and stores its results in the
 * buffers given to the submit.  So a producer gathers batch i+1 while batch i crosses PCIe and
 * runs.  Windows are 48 B when every frame longer than 48 B has IHL <= 7 (64 or 80 B otherwise).
 * Batches of one handle are classified in submit order.  A submit into a slot whose batch was
 * not waited for completes that batch first.  Everything a submit names (mbufs, lens, outputs)
 * must stay valid until its wait returns (or the slot is reused).  Replaces a sequence of
 * GroupByProducer::execute calls over host mbufs (operators/group_by.rs:43-55).
 * A batch of at most 2,048 packets takes the direct path: one kernel launch reads the staged windows
 * (or, zero-copy, the offsets and frames) out of host memory and stores its results there, with no
 * DMA copy either way; larger batches are copied H2D / D2H around the kernels.  A direct batch whose
 * frames longer than 40 B all have IHL <= 5 is staged as 32-B windows (frame bytes 8..39: everything
 * the parse reads once the MACs are swapped), a third fewer bytes over PCIe.
 */
#define NBG_HOST_SLOTS 8
int nbg_maglev_host_submit(nbg_maglev* h, uint8_t* const* pkt_ptrs, const uint16_t* lens, uint64_t n,
                           uint32_t flags, uint16_t* backend_out, uint32_t* perm_out, uint32_t* counts_out,
                           uint64_t* ticket);
int nbg_maglev_host_wait(nbg_maglev* h, uint64_t ticket);
/* Non-blocking: *done = 1 when batch `ticket`'s kernels and copies have finished (its host_wait then
 * returns without waiting on the GPU), 0 otherwise.  A producer that keeps several batches in flight
 * polls the oldest between its scheduler's other tasks instead of blocking in host_wait. */
int nbg_maglev_host_query(nbg_maglev* h, uint64_t ticket, int* done);

/*
 * Zero-copy host path: register a host memory region (a DPDK mempool's hugepage memory, as
 * rte_extmem_register / rte_dev_dma_map would map it for a NIC) once, so that the GPU reads the
 * header windows straight out of the mbufs and writes the MAC swap back into them over PCIe.
 * Then nbg_maglev_classify_device_ex(h, dev_base, d_off, d_len, ...) classifies a burst with
 * d_off[i] = (mbuf data address - base) (u32: regions below 4 GiB) and d_len[i] = data_len, both
 * in HBM; pass NBG_OWNED_WINDOWS (mbuf data rooms are >= 2 KiB) and NBG_WB_PARTIAL (only the
 * 16 B holding the MACs cross PCIe back).  No host thread touches a packet.  *dev_base receives
 * the device address of base.  nbg_host_unregister(base) before the memory is freed.
 * nbg_maglev_host_submit / nbg_maglev_classify_host take this path by themselves when every frame
 * of a batch (and the 64 B from its start) lies in one registered region of the handle's device.
 */
int nbg_host_register(void* base, uint64_t bytes, int device, uint8_t** dev_base);
int nbg_host_unregister(void* base, int device);

/*
 * The host CPUs local to a device (its PCI function's local_cpulist in sysfs, in the kernel's order:
 * the node's physical cores first, then their SMT siblings), for pinning the producer threads that feed
 * it, as a DPDK application puts its lcores on the NIC's socket.  Writes up to cap CPU numbers to cpus
 * and their count to *n (which may exceed cap).  NBG_ENODEV without the device, NBG_EIO when sysfs
 * does not say.  Replaces no reference interface: NetBricks takes its cores from the configuration
 * (config/config_reader.rs), the integration picks them from this list.
 */
int nbg_device_local_cpus(int device, int32_t* cpus, uint32_t cap, uint32_t* n);

/*
 * Host-batch server: one persistent kernel per GPU that takes the direct (<= 2,048-packet) batches of
 * nbg_maglev_host_submit / nbg_maglev_classify_host from every handle attached to it, so a batch costs
 * no kernel launch (one launch per 992-packet batch bounds a multi-pipeline drop-in producer by the
 * GPU's dispatch rate).  Each of `blocks` (0 = 64; at most half the CUs) resident
 * 1024-thread blocks takes the next posted batch from a descriptor ring in pinned host memory,
 * classifies and groups it exactly as the small kernel would, and sets the batch's completion word;
 * results are identical.  Producer threads post concurrently (the calls stay per handle).
 * nbg_maglev_set_host_ring(h, r) attaches a handle (r = NULL detaches; batches already posted
 * complete as before); a batch is launched as before when its handle has no server or the server
 * ended.  The kernel runs on a private stream of the highest priority and ends at
 * nbg_host_ring_stop (every posted batch completes first; NBG_EBUSY while handles are attached), or by
 * itself after idle_ms without a post (0 = 2000 ms; later batches are then launched).  One server per
 * device, not beside a persistent RX ring (nbg_ring_start and nbg_host_ring_start refuse each other
 * with NBG_EBUSY).  nbg_maglev_destroy detaches its handle after its batches completed.
 */
typedef struct nbg_host_ring nbg_host_ring;
int nbg_host_ring_start(int device, uint32_t blocks, uint32_t idle_ms, nbg_host_ring** out);
int nbg_host_ring_stop(nbg_host_ring* r);
int nbg_maglev_set_host_ring(nbg_maglev* h, nbg_host_ring* r);


/* ---- chained NF: test/lpm -> test/maglev (BASELINE config C5) ------------- */

typedef struct nbg_lpm nbg_lpm;

#define NBG_LPM_TBL24_SIZE ((1u << 24) + 1u) /* TBL24_SIZE, test/lpm/src/nf.rs:19 */

/* IPLookup::new + insert(prefix, len, gate) per route + construct_table
 * (test/lpm/src/nf.rs:24-86), uploaded to `device` (tbl24: 32 MiB; tbl_long: the used blocks).
 * prefixes are host-order u32 (u32::from(Ipv4Addr), nf.rs:41); lens in [0, 32].  A later route
 * with the same (prefix, len) replaces an earlier one (HashMap::insert, nf.rs:46).  Routes of
 * one length are applied in ascending prefix order (the reference iterates a HashMap: see
 * DESIGN.md).  NBG_EINVAL where the reference would panic (a fill past the end of a table). */
int nbg_lpm_create(const uint32_t* prefixes, const uint8_t* lens, const uint16_t* gates, uint64_t n, int device,
                   nbg_lpm** out);
void nbg_lpm_destroy(nbg_lpm* t);

/* IPLookup::lookup_entry (nf.rs:88-98) for n host-order IPv4 addresses in HBM -> u16 gates. */
int nbg_lpm_lookup_device(nbg_lpm* t, const uint32_t* d_ips, uint64_t n, uint16_t* d_gate, void* stream);

/*
 * The chain `lpm(ReceiveBatch) -> maglev(...)`: per packet, test/lpm's pipeline
 * (parse::<MacHeader> -> transform(swap_addresses) -> parse::<IpHeader> ->
 * group_by(lpm_groups, lookup_entry(src)), test/lpm/src/nf.rs:212-228) and then test/maglev's
 * (nf.rs:92-106), fused in one kernel pass.  The two MAC swaps cancel, so packet bytes are
 * only read.  Outputs:
 *   d_gate     n_pkts u16: lookup_entry(ip.src), or NBG_SENTINEL when lpm cannot parse the
 *              packet (data_len < 14 + 20: the parse_header asserts, interface/packet.rs:392-399)
 *   d_backend  n_pkts u16: the Maglev backend, or NBG_SENTINEL when either NF would panic
 *              (lpm: unparseable or gate >= lpm_groups, the group index panic of
 *              operators/group_by.rs:48; maglev: as nbg_maglev_classify_device)
 *   d_perm / d_counts  grouped by backend as nbg_maglev_classify_device (input order inside a
 *              group; the reference's cross-group merge order after lpm is scheduler-defined)
 * flags: NBG_OWNED_WINDOWS | NBG_DEFER_GROUP (NBG_SWAP_MACS is ignored: the swaps cancel).
 */
int nbg_chain_lpm_maglev_device(nbg_maglev* mg, nbg_lpm* lpm, uint32_t lpm_groups, uint8_t* d_pkts,
                                const uint32_t* d_off, const uint16_t* d_len, uint32_t stride, uint16_t fixed_len,
                                uint64_t n_pkts, uint32_t flags, uint16_t* d_gate, uint16_t* d_backend,
                                uint32_t* d_perm, uint32_t* d_counts, void* stream);

/* The chain over several descriptor batches in one launch of each kernel (nbg_desc_batch, as
 * nbg_maglev_classify_desc_multi; every batch's d_gate is required).  Each batch's gate / backend /
 * perm / counts are those of nbg_chain_lpm_maglev_device on that batch alone. */
int nbg_chain_lpm_maglev_multi(nbg_maglev* mg, nbg_lpm* lpm, uint32_t lpm_groups, const nbg_desc_batch* batches,
                               uint32_t n_batches, uint32_t flags, void* stream);

const char* nbg_last_error(void);

/* ---- host-only helpers (no GPU needed) ---------------------------------- */

/* The product's own LPM builder (what nbg_lpm_create uploads), for tests: tbl24 has
 * NBG_LPM_TBL24_SIZE entries; tbl_long receives *long_used (<= long_cap) entries. */
int nbg_lpm_build_host(const uint32_t* prefixes, const uint8_t* lens, const uint16_t* gates, uint64_t n,
                       uint16_t* tbl24, uint16_t* tbl_long, uint64_t long_cap, uint64_t* long_used);

/* The product's own LUT builder (what nbg_maglev_create uploads), for tests. */
int nbg_lut_build_host(const char* const* names, const uint32_t* name_lens, uint32_t n_backends,
                       uint64_t table_size, uint16_t* out);

/* Synthetic trace (DESIGN.md "Synthetic traces"): frame layout then bytes.
 * mode: 0 = fixed 60-B UDP frames in 64-B slots, 1 = IMIX 7:4:1 of 60/572/1496-B frames
 * at 64-B aligned offsets.  nbg_trace_layout fills off/len (n entries each) and
 * returns the buffer size in bytes. */
uint64_t nbg_trace_layout(uint64_t n, int mode, uint64_t seed, uint32_t* off, uint16_t* len);

#define NBG_TRACE_UNIQUE 0x1u  /* every packet a new flow */
/* Fill buf with n frames described by off/len; flows drawn from n_flows random 5-tuples. */
int nbg_trace_fill(uint8_t* buf, const uint32_t* off, const uint16_t* len, uint64_t n, uint64_t seed,
                   uint32_t n_flows, uint32_t flags);

#ifdef __cplusplus
}
#endif

#endif /* NBGPU_H */

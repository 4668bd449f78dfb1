/*
 * mte.h — C-ABI of the MI355X batched sequence-merge engine (libmte.so).
 *
 * The engine replays *sequenced* merge-tree messages for many independent
 * documents at once, as an observer client would (every message is remote),
 * and — for documents declared MTE_DOC_LOCAL_CLIENT — as a client that sends:
 * its local ops (MTE_F_LOCAL) and the acks of their sequenced messages
 * (MTE_OP_ACK) interleaved with the remote messages it receives.
 * It replaces, for that path, the following reference interfaces
 * (paths relative to /root/reference/packages/dds/merge-tree/src/):
 *
 *   Client.applyMsg(msg, local=false)        client.ts:918-935
 *     -> Client.applyRemoteOp                client.ts:862-889
 *        -> applyInsertOp / applyRemoveRangeOp / applyAnnotateRangeOp
 *                                            client.ts:470-505 / 405-428 / 435-463
 *        -> MergeTree.insertSegments         mergeTree.ts:1394-1422
 *        -> MergeTree.markRangeRemoved       mergeTree.ts:1908-2000
 *        -> MergeTree.annotateRange          mergeTree.ts:1864-1906
 *     -> Client.updateSeqNumbers / setMinSeq client.ts:937-945, mergeTree.ts:1077-1093
 *   Read-out: TestClient.getText             test/testClient.ts:148-150
 *             Client.getLength               client.ts:1161
 *             Client.getPropertiesAtPosition client.ts:1133-1141
 *
 * Conventions: every function returns an int status (0 = MTE_OK, < 0 = error,
 * never an exception or longjmp across the ABI).  Input buffers are copied
 * before the call returns, so the caller may free them.  Outputs go to caller
 * buffers (query-size-then-fill where sizes are data dependent).  One mte_ctx
 * drives one HIP device; a ctx is not thread-safe, different ctxs are
 * independent (one per process / GPU).  No torch or HIP types appear here.
 */
#ifndef MTE_H_
#define MTE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MTE_ABI_VERSION 1

/* Property key planes held per segment (host interns key strings to 0..n_keys-1). */
#define MTE_MAX_KEYS 8
/* Distinct short client ids per document (removedClientIds is a bitmask):
 * MTE_MAX_CLIENTS on the flat passes, MTE_MAX_CLIENTS_TREE in documents the
 * HBM tree pass replays (MTE_DOC_LOCAL_CLIENT, MTE_DOC_TREE), which hold the
 * mask's upper half in a plane of their own.  A host recycles a short id once
 * the collab window's minSeq passed every seq its client used, so these bound
 * the clients sending inside one window, not a document's clients.  MTE_OP_REF
 * records (b = 2) and mte_seg.removers take ids < MTE_MAX_CLIENTS. */
#define MTE_MAX_CLIENTS 32
#define MTE_MAX_CLIENTS_TREE 64

/* ---- status codes ---------------------------------------------------------
 * Where the reference raises an assert with a hex code, the equivalent code is
 * noted (common-utils assert(cond, 0xNNN)).                                  */
#define MTE_OK 0
#define MTE_E_INVALID_ARG (-1)
#define MTE_E_NO_DEVICE (-2)   /* no HIP device / HIP runtime error at create   */
#define MTE_E_HIP (-3)         /* HIP runtime error (see mte_last_error)        */
#define MTE_E_CAPACITY (-4)    /* doc exceeded its segment capacity             */
#define MTE_E_SEQ_ORDER (-5)   /* seq <= currentSeq          (0x030, 0x038)     */
#define MTE_E_MSN_ORDER (-6)   /* msn < window minSeq        (0x031, 0x04f)     */
#define MTE_E_MSN_GT_SEQ (-7)  /* msn > seq                  (0x039, 0x04e)     */
#define MTE_E_INSERT_FAILED (-8) /* "MergeTree insert failed" mergeTree.ts:1666-1672 */
#define MTE_E_UNSUPPORTED (-9) /* op shape outside the engine (combiningOp other
                                  than rewrite, local/ack ops without
                                  MTE_DOC_LOCAL_CLIENT)                        */
#define MTE_E_STATE (-10)      /* call out of order (e.g. run before submit)    */
#define MTE_E_OOM (-11)        /* device or host allocation failed              */
#define MTE_E_CLIENT_RANGE (-12) /* short client id >= MTE_MAX_CLIENTS          */

/* ---- op records ----------------------------------------------------------- */
/* MergeTreeDeltaType, ops.ts:43-48.  NOOP = a sequenced message that is not an
 * "op" (or an insert without seg): it still advances currentSeq / minSeq
 * (client.ts:922, 934).  GROUP ops (ops.ts:121-124) are flattened by the host
 * into consecutive records with the same seq; only the last carries MSG_END.  */
#define MTE_OP_INSERT 0
#define MTE_OP_REMOVE 1
#define MTE_OP_ANNOTATE 2
#define MTE_OP_NOOP 3
/* The sequenced message of an op this document's own (local) client sent:
 * Client.applyMsg(msg) with msg.clientId == the local client -> ackPendingSegment
 * (client.ts:925-928, mergeTree.ts:1278-1331, mergeTreeNodes.ts:475-503).  The
 * pending segment groups of localSeq pos1 .. pos2 (FIFO, so always the oldest
 * ones) take seq as their insert / removal seq and their pending property keys
 * stop blocking remote annotates; then the window update as for any message.
 * Only in MTE_DOC_LOCAL_CLIENT documents.                                    */
#define MTE_OP_ACK 4
/* Client.rollback of the document's own latest pending op (client.ts:396-398
 * -> MergeTree.rollback, mergeTree.ts:2005-2083), which is then never sent:
 * seq = that op's localSeq, pos1 = its type.  A rolled-back insert becomes a
 * removed segment of seq and removedSeq UniversalSequenceNumber (0), gone for
 * every view; a rolled-back remove restores its segments.  A rolled-back
 * annotate (a = its group slot, see MTE_ANNOTATE_SLOTS; pos2 = the number of
 * MTE_OP_RBKEY records that follow it) puts back, on every segment of its
 * group, the previous value of each key it set (the group's previousProps,
 * mergeTree.ts:2056-2072, segmentPropertiesManager.ts:63-151): the value of
 * the latest older pending annotate of the segment's groups that set the key,
 * else the value the key had before the first pending annotate set it.  A
 * segment of the group removed since stops the document with
 * MTE_E_UNSUPPORTED (the reference would re-annotate the range after it).
 * Only in MTE_DOC_LOCAL_CLIENT documents.                                    */
#define MTE_OP_ROLLBACK 5
/* Client.regeneratePendingOp for reconnection (client.ts:972-1002 ->
 * resetPendingDeltaToOps :788-860): a local record with seq = the localSeq L of
 * a pending op and pos1 = its type.  The text does not change; it reports,
 * as MTE_DELTA_REGEN | type delta records, one per segment of L's segment group
 * in document order, the op that re-sends that segment: its position in the
 * view at localSeq L (findReconnectionPosition :709-713 -> getPosition with
 * localSeq: leaves by localNetLength, mergeTree.ts:575-593 -- acked text plus
 * own pending inserts up to L, minus acked removals and own pending removals
 * up to L -- blocks by the reference's local partial lengths, see MTE_OP_REF
 * b = 4) and its cachedLength.
 *   insert: every segment L inserted (`removed` holds its text offset, whose
 *     difference from the lowest of the group is the segment's offset in the
 *     op's text);
 *   remove: every segment L removes that no remote remove overtook;
 *   annotate: every segment L visited (a = the annotate's group slot, see
 *     MTE_OP_ANNOTATE below) that is not removed, or only by a pending local
 *     remove.
 * A member that re-sends nothing (a removal a remote remove overtook, an
 * annotated segment removed since) leaves the group, as :803-852 dequeue it.
 * The host re-sends the ops and keeps the group pending under the same L
 * (acked by MTE_OP_ACK as before).  Only in MTE_DOC_LOCAL_CLIENT documents
 * that record events (MTE_DOC_EVENTS).                                       */
#define MTE_OP_REGEN 6
#define MTE_DELTA_REGEN 0x10u
/* the answer of an MTE_OP_REF record with b = 4 / 5 (pos; len 0) */
#define MTE_DELTA_REBASE 0x20u
/* A local reference of an MTE_DOC_REFS | MTE_DOC_EVENTS document slid off a
 * segment that became removed and acked (slideAckedRemovedSegmentReferences,
 * mergeTree.ts:921-950, after a remote remove or an ack) or came off it for
 * want of a segment to slide to: one record per reference, in the order of the
 * segments it left; pos = the own-view position of that segment, len = the
 * order key of the unit it left once the message is applied (the held units
 * before it, as mte_read_ref_order counts them; -1 if the zamboni took it),
 * removed = the reference's slot, kind = MTE_DELTA_SLIDE | 1 when it moved onto
 * a segment | 2 when that is the end of a preceding one (addAfterTombstones;
 * else offset 0 of a following one, addBeforeTombstones) | its offset in the
 * segment it left << 16 (clamped to 0xffff; a merged leaf's items are one
 * segment, offsets counted from its first unit).  The reference
 * calls the reference's beforeSlide / afterSlide callbacks at each of them
 * (localReference.ts:436-447, 471-480): an interval collection's "changeInterval"
 * events raised mid-op (intervalCollection.ts:1042-1053). */
#define MTE_DELTA_SLIDE 0x40u
/* MTE_DOC_SLIDE_EVENTS documents: after each record that produced
 * MTE_DELTA_SLIDE records, one record per live reference slot, as that record
 * left the document: pos = its position as mte_read_refs reads it (-1
 * detached), or -2 - p for a reference off the string whose segment
 * mte_read_refs_transient still finds at p; len = its order key (as
 * mte_read_ref_order reads it); removed = the slot.  The reference raises the
 * slides' events mid-op (a group op applies its members one after another,
 * client.ts applyRemoteOp), so a host that delivers them after a batch reads
 * positions and order from these, not from the document after the batch. */
#define MTE_DELTA_REFPOS 0x80u
/* MTE_DOC_MAINT_EVENTS documents: one record per segment of a maintenance
 * callback, kind = MTE_DELTA_MAINT | type (MergeTreeMaintenanceType negated,
 * mergeTreeDeltaCallback.ts:24-50): APPEND (the merged segment, then the one
 * appended to it), SPLIT (the two pieces), UNLINK (a tombstone the zamboni
 * unlinks), ACKNOWLEDGED (the pending group an ack sequenced); removed = the
 * segment's index among the callback's, in document order (the order
 * SequenceMaintenanceEvent.ranges sorts them in, sequenceDeltaEvent.ts:
 * 27-60), so index 0 starts a callback; len = the segment's cachedLength when
 * the callback ran; pos = its position in the document's own view once the
 * record is applied (Client.getPosition, client.ts:345-350), -1 when it is no
 * longer in the tree (an appended or unlinked segment).  In record order with
 * the delta ranges: a split before the op's range, an ack's callback after its
 * slides, the zamboni's appends and unlinks last.                            */
#define MTE_DELTA_MAINT 0x100u
#define MTE_MAINT_APPEND 1u
#define MTE_MAINT_SPLIT 2u
#define MTE_MAINT_UNLINK 3u
#define MTE_MAINT_ACK 4u
/* Follows an annotate's MTE_OP_ROLLBACK (a local record): for each key k the
 * rolled-back annotate set (pos1 = k), the older pending annotates that set k
 * too, latest first -- pos2 = its group slot, a = the value id it set, seq =
 * its localSeq -- then one record with pos2 = MTE_ANNOTATE_SLOTS (the value
 * before the first pending annotate, kept per segment).  A segment takes the
 * first candidate whose group it belongs to.                                 */
#define MTE_OP_RBKEY 7
/* Local references (LocalReferenceCollection, localReference.ts:139-567) in an
 * MTE_DOC_REFS document: a local record (MTE_F_LOCAL, seq 0: it takes no
 * localSeq and moves no window) with pos2 = the reference's slot (0 ..
 * mte_set_ref_capacity - 1, assigned by the host) and b one of:
 *   0 create: Client.createLocalReferencePosition(segment, offset, refType)
 *     (client.ts:360-364, mergeTree.ts:2124-2143) on the segment and offset
 *     that getContainingSegment(pos1) finds in the local view
 *     (mergeTree.ts:872-885); a = the ReferenceType flags (ops.ts): Simple (0),
 *     SlideOnRemove (0x40), StayOnRemove (0x80) or Transient (0x100), plus
 *     any of the label bits; SlideOnRemove with StayOnRemove (or either with
 *     Transient) is MTE_E_INVALID_ARG; pos1 outside the local view
 *     MTE_E_INVALID_ARG.  A Transient reference (localReference.ts:263) stays
 *     on that segment and offset -- never moved, slid or detached -- and
 *     reads as the segment's position, plus the offset unless the segment is
 *     removed, -1 once it is unlinked; local-client documents only (the HBM
 *     tree pass; elsewhere MTE_E_UNSUPPORTED).  b = 2 / 3 with Transient:
 *     MTE_E_UNSUPPORTED.
 *   1 remove: removeLocalReferencePosition (mergeTree.ts:2113-2123).
 *   2 create in a sequenced op's perspective (the interval collection's
 *     remote add / change, intervalCollection.ts:639-658): ref_seq and client
 *     (non-zero) are the op's; getContainingSegment(pos1) in that view, then
 *     getSlideToSegment (mergeTree.ts:893-950); no segment: the reference is
 *     detached.
 *   3 retype: the reference takes type a; if it becomes SlideOnRemove and its
 *     segment is already removed and acked it slides now (ackInterval's
 *     StayOnRemove -> SlideOnRemove conversion, intervalCollection.ts:1805-1902).
 *   4 rebase a position (an interval collection's reconnection,
 *     rebaseLocalInterval intervalCollection.ts:1735-1803 ->
 *     Client.rebasePosition client.ts:755-786): pos1 in the local client's view
 *     at refSeq ref_seq and localSeq a (the pending op's; a <= the document's
 *     localSeq) -> the segment holding it, else the last segment at offset 0;
 *     slid as getSlideToSegment slides (client.ts:1117-1130) if removed and
 *     acked; its position in the view at (currentSeq, a) plus the offset
 *     (findReconnectionPosition :709-713), -1 (DetachedReferencePosition) when
 *     nothing is left to slide to.  Reported as one MTE_DELTA_REBASE event
 *     (pos = the position).  pos2 = 0.
 *   5 re-place a pending interval end on reconnection
 *     (intervalCollection.ts:1782-1799): the reference in slot pos2, if its
 *     segment is removed and acked, moves to the position of its slide target
 *     in the view at (currentSeq, a) -- to what getContainingSegment finds there
 *     (createPositionReference with localSeq :639-658), detached if nothing;
 *     one MTE_DELTA_REBASE event, pos = that position, -1 if it did not move.
 *   b = 4 / 5 only in MTE_DOC_LOCAL_CLIENT | MTE_DOC_EVENTS documents (the
 *   HBM tree pass).  These views -- and MTE_OP_REGEN's positions -- are the
 *   reference's: block lengths from its local partial lengths (partialLengths.ts:
 *   667-700), cached as computeLocalPartials caches them (mergeTree.ts:964-982;
 *   DESIGN.md §4 "Reconnection").
 * The engine slides references as the reference does
 * (slideAckedRemovedSegmentReferences, mergeTree.ts:893-950): when a segment
 * becomes removed and acked -- a remote remove newly removing it or
 * overtaking the local client's pending removal (:1936-1938, 1986-1993), or
 * the ack of the local client's removal (:1302-1304) -- its SlideOnRemove
 * references move to the first following segment that is neither removed and
 * acked nor a pending insert (offset 0), else to the last such preceding one
 * (its last offset), else detach; its Simple references detach; its
 * StayOnRemove references stay on the removed segment.  Positions
 * come from mte_read_refs (referencePositionToLocalPosition,
 * mergeTree.ts:1095-1112).                                                     */
#define MTE_OP_REF 8
/* Relative positions (IRelativePosition, ops.ts:62-76) of the insert, remove
 * or annotate record that follows in the same document (getValidOpRange,
 * client.ts:541-560 -> posFromRelativePos, mergeTree.ts:1369-1392), resolved
 * in that record's own view: its ref_seq and client, the local view for a
 * local record.  a = the property key holding marker ids
 * (reservedMarkerIdKey "markerId"; MTE_NO_PROPS: the context has none), pos1
 * / pos2 = the value ids of relativePos1 / relativePos2's `id` (0: none),
 * seq / ref_seq = their `offset`s (0 when absent), flags MTE_RP_*: which of
 * the two are given and their `before`.  The marker is the first marker
 * segment in document order whose key-a value is the id (idToSegment,
 * mergeTree.ts:490, 597-599; ids are unique per document); with P its
 * position in the view (getPosition, :853-870), the record's position becomes
 * P - offset (before) or P + 1 + offset.  An id no held marker carries gives
 * -1, as the reference's "not found" (a remove or annotate of [-1, -1) does
 * nothing; an insert there stops the document with MTE_E_UNSUPPORTED).  An
 * insert takes relativePos1 only.  Contexts of >= 8192 segments replay such
 * a document of the new length calculation with MTE_E_UNSUPPORTED.         */
#define MTE_OP_RELPOS 9
#define MTE_RP_POS1 0x0100u
#define MTE_RP_BEFORE1 0x0200u
#define MTE_RP_POS2 0x0400u
#define MTE_RP_BEFORE2 0x0800u
#define MTE_REF_SLIDE_ON_REMOVE 0x40u /* ReferenceType.SlideOnRemove             */
#define MTE_REF_STAY_ON_REMOVE 0x80u  /* ReferenceType.StayOnRemove              */
#define MTE_REF_TRANSIENT 0x100u      /* ReferenceType.Transient (b = 0 only)     */
/* Segment groups of pending local annotates (mergeTree.ts:1874-1880): a local
 * annotate record with b = a slot 0..31 marks every segment it visits with
 * that slot (MTE_NO_PROPS: not tracked); an MTE_OP_ACK record's a is the mask
 * of the slots its groups free.  At most 32 tracked annotates are pending at
 * once per document (the host assigns the slots).                           */
#define MTE_ANNOTATE_SLOTS 32

#define MTE_F_MARKER 0x0001u  /* insert spec {marker:{refType}} (mergeTreeNodes.ts:602-609) */
#define MTE_F_MSG_END 0x0002u /* last record of its message: window update follows      */
#define MTE_F_REWRITE 0x0004u /* annotate combiningOp {name:"rewrite"} (segmentPropertiesManager.ts:105-119) */
/* A sequenced annotate with combiningOp "incr" or "consensus": the reference
 * sets each key to combine(op, currentValue, undefined, seq)
 * (segmentPropertiesManager.ts:141, properties.ts:24-62) -- a function of the
 * segment's current value alone -- and ignores pending local keys
 * (shouldModifyKey, :94-102).  The host computes that function over every
 * value the key can hold: the record's propset lists, per key, a header
 * {key, n} and n pairs {old | MTE_COMBINE_PAIR, new} (value ids, 0 = absent);
 * an old value not listed stays.  Only in MTE_DOC_LOCAL_CLIENT and
 * MTE_DOC_TREE documents (the HBM tree pass): MTE_E_UNSUPPORTED otherwise.  A local one (MTE_F_LOCAL,
 * the map made at seq UnassignedSequenceNumber) marks its keys pending and
 * joins its group slot as any local annotate.  On an MTE_OP_ACK record: b is
 * the stamp of a local consensus (updateConsensusProperty, client.ts:646-650,
 * 1083-1090) -- the map made at the ack's seq, applied to the segments of
 * pos2's annotate group (slot in a) whatever their pending keys.             */
#define MTE_F_COMBINE 0x0010u
#define MTE_COMBINE_PAIR 0x80000000u
/* A property value id with this bit set never matches another value id, itself
 * included: matchProperties compares values with !== (properties.ts:66-100), so
 * two segments holding NaN (an incr's result on a number or absent value,
 * properties.ts:24-40) never append-merge in the zamboni (mergeTree.ts:712) or
 * coalesce in a summary (snapshotV1.ts:215, snapshotlegacy.ts:170).  Hosts
 * intern NaN under such an id (id & ~MTE_VALUE_UNEQUAL indexes their value
 * tables as usual). */
#define MTE_VALUE_UNEQUAL 0x40000000u
/* A local op of the document's own client (client 0), not yet sequenced:
 * insertSegmentLocal / removeRangeLocal / annotateRangeLocal (client.ts:131-229)
 * -> insertSegments / markRangeRemoved / annotateRange with seq =
 * UnassignedSequenceNumber (constants.ts:12).  Positions are in the local
 * client's view (every segment it holds, its own pending ones included, minus
 * the removed ones: localNetLength, mergeTree.ts:553-573).  The record's seq is
 * the op's localSeq (collabWindow.localSeq, > 0, strictly increasing per
 * document, < MTE_LOCAL_SEQ_BASE); ref_seq and min_seq are ignored and the
 * window does not move (no MSG_END).  Only in MTE_DOC_LOCAL_CLIENT documents;
 * a local rewrite is MTE_E_UNSUPPORTED.                                       */
#define MTE_F_LOCAL 0x0008u
/* On an MTE_OP_ACK record: the acked message is a regenerated one (an
 * MTE_OP_REGEN record re-sent its localSeqs since they were last sent).
 * resetPendingDeltaToOps gives each re-sent segment an op and a segment group
 * of its own (client.ts:802-857), so the message acks the segments one by one,
 * in document order -- each with the tails split off it since, its own
 * ACKNOWLEDGED maintenance record and its own zamboni pass.                 */
#define MTE_F_REGENERATED 0x0020u
/* Pending (unacked) seqs are held as MTE_LOCAL_SEQ_BASE + localSeq, above any
 * sequenced seq: UnassignedSequenceNumber normalised as in breakTie / nodeLength
 * (mergeTree.ts:1009-1016, 1713-1714).  Sequenced seqs must stay below it.     */
#define MTE_LOCAL_SEQ_BASE 0x40000000

#define MTE_NO_PROPS 0xFFFFFFFFu

/* 32-byte op record (ISequencedDocumentMessage + IMergeTreeDeltaOp, packed).   */
typedef struct mte_op {
  int32_t seq;     /* sequenceNumber                                          */
  int32_t ref_seq; /* referenceSequenceNumber                                 */
  int32_t min_seq; /* minimumSequenceNumber                                   */
  uint8_t type;    /* MTE_OP_*                                                */
  uint8_t client;  /* short client id in first-seen order (client.ts:683-698) */
  uint16_t flags;  /* MTE_F_*                                                 */
  int32_t pos1;    /* insert pos / range start                                */
  int32_t pos2;    /* range end; insert text: UTF-16 unit count; marker: refType */
  uint32_t a;      /* insert text: unit offset in the batch text; annotate: propset */
  uint32_t b;      /* insert: propset of seg.props, or MTE_NO_PROPS            */
} mte_op;

/* A property set: entries[first .. first+count).  value 0 = JSON null (delete
 * the key, segmentPropertiesManager.ts:142-147); other values are host-interned
 * ids of canonical JSON values (equality == matchProperties, properties.ts:66). */
typedef struct mte_prop {
  uint32_t key;
  uint32_t value;
} mte_prop;
typedef struct mte_propset {
  uint32_t first;
  uint32_t count;
} mte_propset;

/* ---- context / documents -------------------------------------------------- */
typedef struct mte_ctx mte_ctx;

typedef struct mte_config {
  int32_t device;        /* HIP device ordinal                                  */
  uint32_t n_keys;       /* property planes per segment, 0..MTE_MAX_KEYS        */
  uint32_t seg_capacity; /* segments per doc kept in HBM (0 = default 1024;
                            >= 8192 adds the chunked big-document pass)       */
  uint32_t flags;        /* reserved, 0                                         */
} mte_config;

/* IMergeTreeOptions.mergeTreeUseNewLengthCalculations, mergeTree.ts:386-399. */
#define MTE_DOC_NEW_LENGTH_CALC 0x1u
/* Round-synchronous stream (the conflict-farm model, test/
 * mergeTreeOperationRunner.ts:149-199): the host declares that the refSeqs of
 * the document's ops never decrease and that each increase reaches the seq of
 * every earlier op.  With the legacy length calculation, insert placement then
 * never depends on the reference's B+tree block edges, so such a
 * document replays on the flat passes instead of the tree pass.  The engine
 * checks the declaration per batch: a batch that breaks it stops the document
 * with MTE_E_UNSUPPORTED before any of the batch's ops (its state stays that of
 * the previous batch).  Ignored with MTE_DOC_NEW_LENGTH_CALC (always flat). */
#define MTE_DOC_ROUND_SYNC 0x2u
/* The document is a collaborating client that sends ops of its own (short
 * client id 0 = collabWindow.clientId): it takes MTE_F_LOCAL records and
 * MTE_OP_ACK messages besides remote ones (the non-observer TestClients of the
 * conflict farm, test/mergeTreeOperationRunner.ts:149-236), in either length
 * calculation.  Such documents replay on the HBM tree pass (the reference's
 * B+tree with its continuePredicate placement, mergeTree.ts:1664, 1790-1791),
 * LDS-resident while they fit.                                               */
#define MTE_DOC_LOCAL_CLIENT 0x4u
/* Record the document's delta events: what MergeTree.mergeTreeDeltaCallback
 * reports after each insert / remove / annotate (mergeTree.ts:1409-1416,
 * 1893-1900, 1978-1985) and SharedString turns into "sequenceDelta" events
 * (sequence.ts:203-211; SequenceEvent.ranges, sequenceDeltaEvent.ts): one
 * mte_delta per affected segment, in document order, at its position in the
 * document's own view right after the op (Client.getPosition, client.ts:345-350).
 * New length-calc documents of remote clients replay on the HBM-streamed pass
 * (refused in contexts of >= 8192 segments), the others on the HBM tree pass.
 * Read with mte_read_deltas.                                                  */
#define MTE_DOC_EVENTS 0x8u
/* The document holds local references (MTE_OP_REF records; mte_read_refs).
 * Requires MTE_DOC_LOCAL_CLIENT.  Each of its markers takes the text offset of
 * its insert record (mte_op.a: the host reserves one unit of the batch text per
 * marker insert), which identifies the marker as a text unit's arena offset
 * identifies that unit.                                                        */
#define MTE_DOC_REFS 0x10u
/* With MTE_DOC_REFS | MTE_DOC_EVENTS: also record the references' slides
 * (MTE_DELTA_SLIDE) and, after each record that slid one, every reference as
 * that record left the document (MTE_DELTA_REFPOS) -- what an interval
 * collection's position-change listeners read mid-op
 * (intervalCollection.ts:1042-1053).  Such a document's event region grows by
 * 2 x the reference slots its MTE_OP_REF records have used for every remote
 * remove and ack record of a batch (a record's slides and snapshot); a host
 * that does not read them leaves the flag clear.                             */
#define MTE_DOC_SLIDE_EVENTS 0x20u
/* With MTE_DOC_EVENTS, on a document of the HBM tree pass (MTE_DOC_LOCAL_CLIENT,
 * MTE_DOC_TREE or the legacy length calculation): also record the
 * merge-tree's maintenance (mergeTreeMaintenanceCallback, mergeTree.ts:695-725,
 * 1313-1320, 1687-1694; SharedString's "maintenance" event,
 * sequence.ts:212-216) as MTE_DELTA_MAINT records.  Opt-in: they take event
 * capacity like the ranges. */
#define MTE_DOC_MAINT_EVENTS 0x40u
/* Replay a new length-calc document without a local client on the HBM tree
 * pass too: the reference's own segmentation (its B+tree, the lazy zamboni's
 * appends), so its delta records are segment-exact -- one range per segment
 * as mergeTreeDeltaCallback reports it, an annotate over a segment removed in
 * the own view with that segment's cachedLength -- where the flat passes'
 * canonical segments can split or join them.  Slower than the flat passes
 * (one wavefront per document); local-client and legacy documents with
 * events replay there anyway. */
#define MTE_DOC_TREE 0x80u

/* Initial document: one text segment inserted before collaboration starts, as
 * the reference replay harness does (client.replay.spec.ts:22-23): seq 0
 * (UniversalSequenceNumber) and clientId -1 (LocalClientId), constants.ts:11,14. */
typedef struct mte_doc_init {
  uint32_t text_off; /* units offset into the load text buffer                */
  uint32_t text_len; /* 0 = empty document                                    */
  uint32_t flags;    /* MTE_DOC_*                                             */
  uint32_t propset;  /* props of the initial segment, or MTE_NO_PROPS          */
  int32_t min_seq;   /* collab window at load (startOrUpdateCollaboration)    */
  int32_t cur_seq;
} mte_doc_init;

/* A segment with its merge info, as a summary holds it and SnapshotLoader
 * restores it (IJSONSegmentWithMergeInfo, snapshotChunks.ts:48-78;
 * snapshotLoader.ts:85-125): seq / client default to UniversalSequenceNumber /
 * NonCollabClient there; here they are explicit.  client -1 stands for both
 * LocalClientId and NonCollabClient (constants.ts:14-15): neither equals a
 * remote short id, which is all the replay asks of it.                      */
#define MTE_NOT_REMOVED 0x7fffffff
typedef struct mte_seg {
  uint32_t text_off;   /* text: unit offset into the mte_load_docs text       */
  uint32_t len;        /* text: units (> 0); marker: 1                        */
  int32_t seq;         /* insert seq (0 = UniversalSequenceNumber)            */
  int32_t removed_seq; /* MTE_NOT_REMOVED or the removal seq                  */
  uint32_t removers;   /* removedClientIds as a short-id bitmask             */
  int32_t client;      /* short client id, or -1                              */
  uint32_t kind;       /* 0 = text, 1 + refType = marker                      */
  uint32_t propset;    /* index into the mte_load_docs propsets, or MTE_NO_PROPS */
} mte_seg;

/* One batch of sequenced ops for all documents of the ctx. */
typedef struct mte_batch {
  uint32_t n_docs;            /* must equal the loaded doc count               */
  const uint64_t* op_offsets; /* n_docs+1: doc d owns ops[op_offsets[d]..[d+1]) */
  const mte_op* ops;          /* per doc in sequence order                     */
  uint64_t n_ops;
  const uint16_t* text; /* UTF-16 payload of inserts (mte_op.a/.pos2)        */
  uint64_t text_units;
  const mte_propset* propsets;
  uint32_t n_propsets;
  const mte_prop* props;
  uint32_t n_props;
} mte_batch;

typedef struct mte_stats {
  uint64_t ops_applied;     /* records applied (NOOPs included)               */
  uint64_t segs_scanned;    /* sum over ops of live segments before the op    */
  uint64_t segs_written;    /* split halves + inserted + marked segments      */
  uint64_t prop_writes;     /* (segment, key) property writes                 */
  uint64_t units_inserted;  /* UTF-16 units inserted                          */
  uint64_t max_segs;        /* max segments held by any doc                   */
  double kernel_ms;         /* device time of the last mte_run (HIP events)   */
  double algo_bytes;        /* sum of B_op of the last run   */
  uint64_t chunk_scanned;   /* chunked pass: chunk slots + summary entries its
                               ops scanned (replaces their S_live in algo_bytes) */
  double round_bytes;       /* chunked pass, round phases: the bytes they had to
                               read and write in the last run (records, planes
                               re-laid out / applied / gathered, sub-op lists),
                               counted with statistics off too               */
} mte_stats;

/* Per-doc read-out (query-size-then-fill).  On input the *_cap fields give the
 * capacity of the caller arrays (0 / NULL = query only); on output the n_*
 * fields give the sizes.  Segments are the visible (non-removed) segments in
 * document order; text is the getText() string (markers contribute no units,
 * MergeTreeTextHelper.ts:49-74).                                              */
typedef struct mte_doc_view {
  int32_t status;  /* 0 or the MTE_E_* that stopped this doc                 */
  int32_t cur_seq; /* collabWindow.currentSeq                               */
  int32_t min_seq; /* collabWindow.minSeq                                   */
  uint32_t length; /* getLength(): visible units incl. markers              */
  uint16_t* text;
  uint32_t text_cap;
  uint32_t n_text;
  uint32_t* seg_len;   /* per visible segment: length                       */
  uint32_t* seg_kind;  /* 0 = text, 1 + refType = marker                    */
  uint32_t* seg_props; /* n_keys values per segment (0 = absent)            */
  uint32_t seg_cap;
  uint32_t n_segs;
} mte_doc_view;

int mte_abi_version(void);
const char* mte_strerror(int code);
/* Build provenance of this library (no reference counterpart): "src=<first 16
 * hex digits of the sha256 of the engine sources it was compiled from
 * (fluidframework_amd/csrc/mte_*.h, mte_*.hip, then include/mte.h, in name
 * order)> arch=gfx950 compiler=<the HIP compiler's version string>", so a host
 * can check that the library it loaded was built from the sources beside it. */
const char* mte_build_info(void);

int mte_create(const mte_config* cfg, mte_ctx** out);
int mte_destroy(mte_ctx* ctx);
const char* mte_last_error(const mte_ctx* ctx);

/* Load (or reload) all documents; resets every doc to its initial state. */
int mte_load_docs(mte_ctx* ctx, uint32_t n_docs, const mte_doc_init* docs,
                  const uint16_t* text, uint64_t text_units,
                  const mte_propset* propsets, uint32_t n_propsets,
                  const mte_prop* props, uint32_t n_props);

/* Replace the loaded content of documents with segment lists (a summary's
 * body, SnapshotLoader.loadBody snapshotLoader.ts:85-130): doc d takes
 * segs[seg_offsets[d] .. seg_offsets[d+1]); a doc with an empty range keeps its
 * mte_load_docs text.  Call after mte_load_docs; mte_reset restores this state.
 * Text offsets and propsets refer to the buffers given to mte_load_docs.     */
int mte_load_segments(mte_ctx* ctx, const uint64_t* seg_offsets, const mte_seg* segs,
                      uint64_t n_segs);

/* Upload one batch (host -> HBM on the ctx stream; returns once the inputs are
 * copied).  Every record is validated on the way; on an error the previously
 * submitted batch is discarded (mte_run then returns MTE_E_STATE).           */
int mte_submit(mte_ctx* ctx, const mte_batch* batch);
/* Enqueue the replay of the submitted batch; returns without waiting. */
int mte_run(mte_ctx* ctx);
/* Wait for the ctx stream; returns the first per-doc error, if any. */
int mte_sync(mte_ctx* ctx);
/* Restore every doc to its loaded state (device side); the batch stays. */
int mte_reset(mte_ctx* ctx);

/* Canonical per-doc digest, 4 x uint64 per doc (see DESIGN.md "Digest"). */
int mte_digest(mte_ctx* ctx, uint64_t* out, uint32_t n_docs);
/* Same digest written to a caller-owned device buffer (for RCCL gathers). */
int mte_digest_device(mte_ctx* ctx, void* device_out, uint32_t n_docs);

int mte_read_doc(mte_ctx* ctx, uint32_t doc, mte_doc_view* view);

/* One delta event range (ISequenceDeltaRange): the record (index in the doc's
 * part of the last batch) whose op caused it, MergeTreeDeltaType (INSERT /
 * REMOVE / ANNOTATE; MTE_DELTA_REGEN | type for the segments an MTE_OP_REGEN
 * record re-sends, positioned as that record describes), the segment's position in the doc's own view right after
 * the op (-1 for a zero-length insert, which links no segment) and its length
 * (cachedLength).  A remove reports only segments it newly removed
 * (removedSegments, mergeTree.ts:1954-1959); an annotate every segment it
 * visited; no event when none (the deltaSegments.length > 0 checks).       */
typedef struct mte_delta {
  uint32_t op;
  uint32_t kind;
  int32_t pos;
  int32_t len;
  uint32_t removed; /* 1: the segment is removed in the doc's own view (an
                       annotate of text another client removed since);
                       MTE_DELTA_REGEN | INSERT records: the text offset    */
} mte_delta;
/* Events of the last mte_run for an MTE_DOC_EVENTS doc (query-size-then-fill:
 * *n gets the count; up to cap are copied).  MTE_E_CAPACITY when the doc
 * produced more than its event capacity (mte_set_event_capacity).            */
int mte_read_deltas(mte_ctx* ctx, uint32_t doc, mte_delta* out, uint64_t cap, uint64_t* n);
/* Event capacity of an MTE_DOC_EVENTS doc per batch: per_op x its records +
 * 256 (default per_op 8); applies from the next mte_submit.                 */
int mte_set_event_capacity(mte_ctx* ctx, uint32_t per_op);

/* Local reference slots per MTE_DOC_REFS document (default 1024).  Set before
 * mte_load_docs; references live until removed or the next mte_load_docs /
 * mte_reset.                                                                   */
int mte_set_ref_capacity(mte_ctx* ctx, uint32_t per_doc);
/* Positions of reference slots [0, n) of doc in its own view after the last
 * mte_run: Client.localReferencePositionToPosition -> MergeTree.
 * referencePositionToLocalPosition (client.ts:376-378, mergeTree.ts:1095-1112):
 * the segment's position (Client.getPosition) plus the offset, 0 on a removed
 * segment; -1 (DetachedReferencePosition) for a detached or unused slot.      */
int mte_read_refs(mte_ctx* ctx, uint32_t doc, int32_t* pos, uint32_t n);
/* As mte_read_refs with every reference Transient, as an interval
 * collection's emitChange reads a changeInterval event's previous interval
 * (intervalCollection.ts:1387-1410; mergeTree.ts:1106-1109): a reference that
 * slid off the string -- its segment removed and acked with no segment to
 * slide to, so slideAckedRemovedSegmentReferences took it off the segment's
 * list but left it pointing there (mergeTree.ts:935-942) -- still gives the
 * position of that segment while the document holds it.                     */
int mte_read_refs_transient(mte_ctx* ctx, uint32_t doc, int32_t* pos, uint32_t n);
/* Document order of reference slots [0, n): the index, among every text unit
 * the document holds (removed segments included), of the unit the reference
 * sits on (a reference that slid off the string: the unit it still points at,
 * while held); -1 for a detached or unused slot.  Two references compare as
 * compareReferencePositions does (referencePositions.ts:81-89: the same
 * segment by offset, else by segment ordinal; detached first) -- the order of
 * an interval collection's tree (intervalCollection.ts:483-520).            */
int mte_read_ref_order(mte_ctx* ctx, uint32_t doc, int64_t* key, uint32_t n);

/* Every segment a document holds — removed ones above minSeq included — with
 * its merge info, in document order: the input of a summary writer
 * (SnapshotV1.extractSegment, snapshotV1.ts:189-265).  Query-size-then-fill
 * like mte_doc_view.  segs[i].text_off indexes `text`, segs[i].propset is
 * MTE_NO_PROPS and the values are in props[i * n_keys ..].                   */
typedef struct mte_seg_list {
  mte_seg* segs;
  uint32_t* props;
  uint64_t seg_cap;
  uint64_t n_segs;
  uint16_t* text;
  uint64_t text_cap;
  uint64_t n_text;
} mte_seg_list;
int mte_read_segments(mte_ctx* ctx, uint32_t doc, mte_seg_list* list);
int mte_doc_status(mte_ctx* ctx, int32_t* out, uint32_t n_docs);
int mte_stats_get(mte_ctx* ctx, mte_stats* out);
/* Statistics accounting (the counters of mte_stats, like the reference's
 * opt-in Client.measureOps, client.ts:71-78) is on by default; with enable = 0
 * the replay kernels are built without the per-op counter updates and
 * mte_stats_get reports zero counts (kernel_ms stays valid). */
int mte_set_stats(mte_ctx* ctx, int enable);

/* ---- Node level: one process per GPU, RCCL over xGMI ----------------------
 * Documents are independent, so the host shards them over the GPUs (one
 * context each) and no collective touches the replay.  These
 * entry points carry what the node-level job needs beside it, over RCCL: a
 * barrier and scalar reductions for timing, and the verification all-gather of
 * every rank's per-document digests.  The reference has no multi-process
 * merge-tree (one Client per document per process); this replaces running
 * those Clients in many processes and comparing their texts.
 *
 * mte_comm_unique_id runs on one rank; the host hands the 128 bytes to the
 * others (any side channel) before every rank calls mte_comm_init.           */
#define MTE_COMM_ID_BYTES 128
#define MTE_COMM_SUM 0
#define MTE_COMM_MAX 1
int mte_comm_unique_id(uint8_t id[MTE_COMM_ID_BYTES]);
int mte_comm_init(mte_ctx* ctx, int world, int rank, const uint8_t id[MTE_COMM_ID_BYTES]);
/* Let another context of this process use src's communicator.  The contexts
 * sharing it hold it by reference count: mte_comm_destroy / mte_destroy of any
 * of them (in any order) releases that context's reference, and the last one
 * destroys the communicator.  Collectives of the contexts sharing one
 * communicator must not overlap in time.                                     */
int mte_comm_share(mte_ctx* ctx, const mte_ctx* src);
/* The context's world size and rank (1 / 0 without a communicator).         */
int mte_comm_world(const mte_ctx* ctx, int32_t* world, int32_t* rank);
int mte_comm_barrier(mte_ctx* ctx);
/* In place, across ranks: op = MTE_COMM_SUM / MTE_COMM_MAX. */
int mte_comm_allreduce_f64(mte_ctx* ctx, double* value, int op);
/* Digests of this context's documents, padded with zero rows to docs_per_rank
 * (>= n_docs, equal on all ranks), gathered in rank order into `out` (host,
 * world * docs_per_rank * 4 uint64; out_cap = the uint64 elements `out` holds,
 * MTE_E_INVALID_ARG when that is fewer).                                      */
int mte_comm_gather_digests(mte_ctx* ctx, uint64_t* out, uint64_t out_cap, uint32_t docs_per_rank);
int mte_comm_destroy(mte_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* MTE_H_ */

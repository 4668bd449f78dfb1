"""Host half of Client.applyMsg: turn ISequencedDocumentMessage objects into
32-byte op records for the device engine.

Reference behaviour mirrored here (packages/dds/merge-tree/src):
  * short client ids in first-seen order, the observer's own id first
    (Client.getOrAddShortClientId / startOrUpdateCollaboration,
    client.ts:683-698, 1163-1183); every message registers its sender
    (client.ts:920), "op" or not;
  * only type "op" messages carry a merge-tree op; all messages advance
    currentSeq / minSeq (client.ts:922-934) -> non-op messages become NOOP
    records;
  * GROUP ops apply their members in order with the same sequenced message
    (client.ts:876-884) -> one record per member, MSG_END on the last;
  * insert specs: string -> text, {text, props} -> text with props,
    {marker:{refType}, props} -> marker (test/testClient.ts:32-44,
    textSegment.ts:40-48, mergeTreeNodes.ts:602-609); an insert without seg
    is a no-op (client.ts:481-487);
  * annotate props: null deletes, anything else sets; combiningOp "rewrite"
    is supported, other combining ops are rejected;
  * a document whose own client sends (DocClients(local=True)): its local ops
    become MTE_F_LOCAL records numbered by collabWindow.localSeq
    (client.ts:131-229, mergeTree.ts:1590-1625), and the sequenced message of
    each comes back as an MTE_OP_ACK record for the oldest pending localSeqs
    (client.ts:925-928 -> ackPendingSegment, mergeTree.ts:1278-1331).
Property keys are interned to plane indices and values to ids of their
canonical JSON (sorted keys), so id equality == matchProperties
(properties.ts:66-100).
"""
import json

import numpy as np

from .abi import (COMBINE_PAIR, MTE_VALUE_UNEQUAL, F_COMBINE, F_LOCAL, F_REGENERATED, F_MARKER, F_MSG_END, F_REWRITE, LOCAL_SEQ_BASE, MTE_E_CAPACITY, MTE_E_CLIENT_RANGE,
                  MTE_E_INVALID_ARG, MTE_E_STATE, MTE_E_UNSUPPORTED, MTE_MAX_CLIENTS, MTE_MAX_CLIENTS_TREE, NO_PROPS, OP_ACK, OP_ROLLBACK,
                  OP_REGEN, OP_RBKEY, OP_REF, OP_RELPOS, RP_BEFORE1, RP_BEFORE2, RP_POS1, RP_POS2,
                  ANNOTATE_SLOTS, REF_SLIDE_ON_REMOVE, REF_STAY_ON_REMOVE,
                  REF_TRANSIENT,
                  OP_ANNOTATE, OP_DTYPE, OP_INSERT, OP_NOOP, OP_REMOVE, PROP_DTYPE, PROPSET_DTYPE,
                  MergeTreeError)

INSERT, REMOVE, ANNOTATE, GROUP = 0, 1, 2, 3  # MergeTreeDeltaType, ops.ts:43-48
I32_MIN, I32_MAX = -(1 << 31), (1 << 31) - 1
MARKER_ID_KEY = "markerId"  # reservedMarkerIdKey (mergeTreeNodes.ts)


def canonical_json(v) -> str:
    return json.dumps(v, sort_keys=True, separators=(",", ":"), ensure_ascii=False)


def utf16_units(s: str) -> np.ndarray:
    """JS strings are UTF-16 code-unit arrays (textSegment.ts:52-55)."""
    return np.frombuffer(s.encode("utf-16-le"), dtype="<u2").copy()


def units_to_str(u) -> str:
    return np.asarray(u, dtype="<u2").tobytes().decode("utf-16-le", errors="surrogatepass")


COMBINE_DOMAIN_MAX = 4096  # distinct values of one key a combining op's value map may cover


class Interner:
    """Key -> plane index, canonical JSON value -> id (0 is reserved for null)."""

    def __init__(self, n_keys: int):
        self.n_keys = n_keys
        self.keys = {}
        self.key_names = []
        self.values = {}
        self.value_json = [None]
        # per value id, the keys it was ever given (bit k), and per key how many:
        # the combining ops' domain, one byte per value (n_keys <= 8) as the Node
        # packer keeps it; a combining op over a key given more than
        # COMBINE_DOMAIN_MAX values is refused (its value map would be that long)
        self.key_mask = bytearray(256)
        self.key_count = [0] * max(1, n_keys)

    def note_value(self, k: int, vid: int):
        """value id `vid` was given to key `k`."""
        x = vid & ~MTE_VALUE_UNEQUAL
        if x >= len(self.key_mask):
            self.key_mask.extend(bytes(max(x + 1, 2 * len(self.key_mask)) - len(self.key_mask)))
        if not self.key_mask[x] & (1 << k):
            self.key_mask[x] |= 1 << k
            self.key_count[k] += 1

    def domain_of(self, k: int):
        """The value ids key k was ever given, ascending (NaN's with its flag)."""
        if self.key_count[k] > COMBINE_DOMAIN_MAX:
            raise MergeTreeError(MTE_E_UNSUPPORTED, f"combiningOp over key {self.key_names[k]!r}, given "
                                 f"{self.key_count[k]} distinct values (> {COMBINE_DOMAIN_MAX})")
        b = 1 << k
        return [x | (MTE_VALUE_UNEQUAL if self.value_json[x] == "NaN" else 0)
                for x in range(1, min(len(self.value_json), len(self.key_mask))) if self.key_mask[x] & b]

    def kv(self, name: str, v):
        """(key, value id) of one property, noting the value under its key."""
        k, vid = self.key(name), self.value(v)
        if vid:
            self.note_value(k, vid)
        return k, vid

    def key(self, name: str) -> int:
        k = self.keys.get(name)
        if k is None:
            if len(self.key_names) >= self.n_keys:
                raise MergeTreeError(MTE_E_UNSUPPORTED,
                                     f"more than n_keys={self.n_keys} property keys ({name!r})")
            k = len(self.key_names)
            self.keys[name] = k
            self.key_names.append(name)
        return k

    def value(self, v) -> int:
        if v is None:
            return 0
        cj = canonical_json(v)
        i = self.values.get(cj)
        if i is None:
            i = len(self.value_json)
            if cj == "NaN":  # matchProperties: NaN !== NaN (include/mte.h MTE_VALUE_UNEQUAL)
                i |= MTE_VALUE_UNEQUAL
            self.values[cj] = i
            self.value_json.append(cj)
        return i

    def json_of(self, vid: int) -> str:
        """canonical JSON of a value id"""
        return self.value_json[vid & ~MTE_VALUE_UNEQUAL]

    def decode_props(self, planes) -> dict:
        out = {}
        for k, vid in enumerate(planes):
            if vid:
                out[self.key_names[k]] = json.loads(self.json_of(int(vid)))
        return out


class PropTable:
    """Property sets of one batch (mte_propset / mte_prop arrays)."""

    def __init__(self, interner: Interner):
        self.interner = interner
        self.sets = []
        self.entries = []
        self.comb_of = {}  # a combining set's index -> (props, combiningOp)

    def add(self, props: dict) -> int:
        if props is None:
            return NO_PROPS
        if not isinstance(props, dict):
            raise MergeTreeError(MTE_E_INVALID_ARG, "props must be an object")
        first = len(self.entries)
        for name, v in props.items():
            self.entries.append(self.interner.kv(name, v))
        self.sets.append((first, len(self.entries) - first))
        return len(self.sets) - 1

    def add_combining(self, props: dict, comb: dict, seq: int) -> int:
        """The property set of an annotate with combiningOp incr / consensus: per
        key a header (key, n) and n pairs (old value id | MTE_COMBINE_PAIR, new
        value id) -- the map combine(comb, old, undefined, seq) makes of every
        value the key can hold (segmentPropertiesManager.ts:141: the op's own
        value is never read), old values it leaves alone omitted, 0 = absent."""
        if not isinstance(props, dict):
            raise MergeTreeError(MTE_E_INVALID_ARG, "props must be an object")
        it = self.interner
        first = len(self.entries)
        for name in props:
            k = it.key(name)
            dom = sorted(it.domain_of(k)) + [0]
            pairs = []
            for old in dom:
                cur = _ABSENT if old == 0 else json.loads(it.json_of(old))
                new = combine_value(comb, cur, seq)
                nid = 0 if new is _ABSENT else it.value(new)
                if nid != old:
                    pairs.append((old | COMBINE_PAIR, nid))
            for _, nid in pairs:
                if nid:
                    it.note_value(k, nid)
            self.entries.append((k, len(pairs)))
            self.entries.extend(pairs)
        self.sets.append((first, len(self.entries) - first))
        self.comb_of[len(self.sets) - 1] = (props, comb)
        return len(self.sets) - 1

    def arrays(self):
        ps = np.array(self.sets, dtype=PROPSET_DTYPE) if self.sets else np.zeros(0, PROPSET_DTYPE)
        pe = np.array(self.entries, dtype=PROP_DTYPE) if self.entries else np.zeros(0, PROP_DTYPE)
        return ps, pe


_ABSENT = object()  # a key the segment does not have (JS undefined)
_NAN = float("nan")


def _js_num(x) -> str:
    """Number.prototype.toString (ECMA-262 Number::toString, radix 10): the
    shortest round-trip digits (Python's repr finds the same ones), written
    plain when the decimal exponent n is in (-6, 21], else as d.ddde+-n-1."""
    import decimal
    if x != x:
        return "NaN"
    x = float(x)
    if x in (float("inf"), float("-inf")):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0:
        return "0"
    if x < 0:
        return "-" + _js_num(-x)
    t = decimal.Decimal(repr(x)).normalize().as_tuple()
    digits = "".join(str(d) for d in t.digits)
    k = len(digits)
    n = k + t.exponent  # x = 0.digits x 10^n
    if k <= n <= 21:
        return digits + "0" * (n - k)
    if 0 < n <= 21:
        return digits[:n] + "." + digits[n:]
    if -6 < n <= 0:
        return "0." + "0" * (-n) + digits
    e = n - 1
    sign = "+" if e >= 0 else "-"
    return (digits if k == 1 else digits[0] + "." + digits[1:]) + "e" + sign + str(abs(e))


def _js_str(v) -> str:
    """String(v) for a JSON value (arrays join their elements, null -> "")."""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, float)):
        return _js_num(v)
    if isinstance(v, str):
        return v
    if isinstance(v, list):
        return ",".join("" if e is None else _js_str(e) for e in v)
    return "[object Object]"


def _js_truthy(v) -> bool:
    if v is _ABSENT or v is None or v is False or v == "":
        return False
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return v == v and v != 0
    return True


def _utf16(s: str) -> bytes:
    return s.encode("utf-16-be")


def combine_value(comb: dict, cur, seq: int):
    """combine(combiningInfo, currentValue, undefined, seq) (properties.ts:24-62)
    with JS semantics: incr adds undefined -- a number, boolean, null or
    absent value becomes NaN, a string s becomes s + "undefined" (an array or
    object its String() form + "undefined") -- then a truthy minValue replaces
    a string below it (both strings: UTF-16 order; otherwise the comparison is
    on NaN and false); consensus makes {value: undefined, seq} (JSON {"seq":
    seq}) of an absent value and stamps the seq of an object whose seq is -1
    (in place in the reference: see DESIGN.md on aliasing), other values stay."""
    name = comb.get("name")
    if cur is _ABSENT and "defaultValue" in comb:
        cur = comb["defaultValue"]
    if name == "incr":
        if cur is _ABSENT or cur is None or isinstance(cur, (bool, int, float)):
            cur = _NAN
        else:
            cur = _js_str(cur) + "undefined"
        mv = comb.get("minValue", _ABSENT)
        if _js_truthy(mv) and isinstance(cur, str):
            pm = mv if isinstance(mv, str) else (_js_str(mv) if isinstance(mv, (list, dict)) else None)
            if pm is not None and _utf16(cur) < _utf16(pm):
                cur = mv
        return cur
    if name == "consensus":
        if cur is _ABSENT or cur is None:
            return {"seq": seq}
        if isinstance(cur, dict) and cur.get("seq") == -1:
            return {**cur, "seq": seq}
        return cur
    raise MergeTreeError(MTE_E_UNSUPPORTED, f"combiningOp {name!r}")


DEFAULT_REF_CAPACITY = 1024  # mte_set_ref_capacity's default (include/mte.h)


def _ref_slot(clients) -> int:
    """The next reference slot of a document: a removed one first, else a new one,
    which must stay below the context's per-document capacity (clients.ref_cap)."""
    if clients.ref_free:
        return clients.ref_free.pop()
    if clients.ref_next >= clients.ref_cap:
        raise MergeTreeError(MTE_E_CAPACITY, f"more than {clients.ref_cap} live local references in one "
                             "document (mte_set_ref_capacity)")
    clients.ref_next += 1
    return clients.ref_next - 1


class DocClients:
    """Per-document long -> short client id map (client.ts:683-698).

    The reference numbers clients forever; the engine's short ids are MTE_MAX_CLIENTS
    slots (the removers bitmask is 32 bits), MTE_MAX_CLIENTS_TREE in the documents the
    HBM tree pass replays (local-client and MTE_DOC_TREE ones: 64 bits).  A slot is recycled for a new client once the
    collab window's minSeq has passed every seq its client used: from then on each of its
    segments has seq <= minSeq <= refSeq (visible to every perspective whoever inserted
    it, mergeTree.ts:1003-1054) and each segment it removed has removedSeq <= minSeq and
    was compacted at that window advance (mergeTree.ts:1077-1093), so the slot number
    decides no visibility rule any more (every later op has refSeq >= minSeq: the
    sequencer's MSN is the minimum of the clients' refSeqs).  Only clients active
    inside the window need distinct slots."""

    NEVER = I32_MAX  # slot held for good (observer, ids registered without a seq)

    def __init__(self, observer_id: str, min_seq: int = 0, local: bool = False, ref_cap: int = DEFAULT_REF_CAPACITY,
                 tree: bool = False):
        self.observer = observer_id
        # an MTE_DOC_TREE document (the HBM tree pass without a local client):
        # it takes sequenced combining ops too
        self.tree = tree
        self.max_clients = MTE_MAX_CLIENTS_TREE if (local or tree) else MTE_MAX_CLIENTS
        self.ids = {observer_id: 0}
        self.last = {0: self.NEVER}  # slot -> highest seq its client used
        self.min_seq = min_seq       # the window's minSeq before the next message
        # local client (MTE_DOC_LOCAL_CLIENT documents): collabWindow.localSeq and
        # the (first, last) localSeqs of each unacked local message, oldest first
        # (MergeTree.pendingSegments, mergeTree.ts:1333-1355)
        self.local = local
        self.local_seq = 0
        self.pending = []
        self.pending_types = []  # the record types of each pending message (rollback)
        # segment groups of pending local annotates: localSeq -> group slot
        # (MTE_ANNOTATE_SLOTS, include/mte.h); an annotate made while all are
        # taken is not tracked and cannot be regenerated
        self.ann_slot = {}
        # acks of such untracked annotates: the engine cannot tell their
        # segments (no ACKNOWLEDGED maintenance record, MTE_DOC_MAINT_EVENTS)
        self.untracked_acks = 0
        # the first localSeqs of the pending messages regenerated since sent
        # (their acks carry F_REGENERATED)
        self.regenerated = set()
        # the keys -> value ids each pending local annotate set (its rollback
        # puts the older values back), and the annotates whose rollback the
        # engine cannot restate exactly (see BatchBuilder.add_rollback)
        self.ann_props = {}
        # the pending local incr / consensus annotates: localSeq -> (props, combiningOp)
        self.ann_comb = {}
        self.no_rollback = set()
        # local reference slots (MTE_DOC_REFS documents): the next unused one and
        # the removed ones, reused first
        self.ref_next = 0
        self.ref_free = []
        # the context's reference slots per document (mte_set_ref_capacity); a slot
        # at or past it would fail the whole batch at mte_submit, so the packer
        # refuses the reference for this document alone (EngineBase.doc_clients
        # passes the engine's capacity)
        self.ref_cap = ref_cap

    def short(self, long_id, seq=None) -> int:
        i = self.ids.get(long_id)
        if i is None:
            i = self._free_slot()
            if i >= self.max_clients:
                return i  # the caller raises MTE_E_CLIENT_RANGE
            self.ids[long_id] = i
            self.last[i] = self.NEVER if seq is None else seq
        elif seq is not None and self.last[i] != self.NEVER:
            self.last[i] = max(self.last[i], seq)
        return i

    def _free_slot(self) -> int:
        used = set(self.ids.values())
        for slot in range(1, self.max_clients):
            if slot not in used:
                return slot
        seq, slot = min((self.last[v], v) for v in used if v != 0)
        if seq > self.min_seq:
            return self.max_clients
        del self.ids[next(k for k, v in self.ids.items() if v == slot)]
        return slot

    def advance(self, msn: int):
        """After a message: the window's minSeq becomes max(minSeq, msn) (client.ts:937-945)."""
        if msn > self.min_seq:
            self.min_seq = msn


def _check_i32(v, what):
    if not isinstance(v, int) or isinstance(v, bool) or v < I32_MIN or v > I32_MAX:
        raise MergeTreeError(MTE_E_INVALID_ARG, f"{what}={v!r} is not an int32")
    return v


class BatchBuilder:
    """Collects messages for n_docs documents and emits one mte_batch."""

    def __init__(self, n_docs: int, interner: Interner):
        self.n_docs = n_docs
        self.interner = interner
        self.props = PropTable(interner)
        self.ops = [[] for _ in range(n_docs)]
        self.text = []
        self.text_units = 0

    def _text(self, s: str):
        u = utf16_units(s)
        off = self.text_units
        self.text.append(u)
        self.text_units += len(u)
        return off, len(u)

    def add_message(self, doc: int, clients: DocClients, msg: dict):
        """Client.applyMsg(msg, local=false) for one document (client.ts:918-935)."""
        sender = msg.get("clientId")
        seq = _check_i32(msg["sequenceNumber"], "sequenceNumber")
        ref = _check_i32(msg.get("referenceSequenceNumber", 0), "referenceSequenceNumber")
        msn = _check_i32(msg["minimumSequenceNumber"], "minimumSequenceNumber")
        # a recycled slot is only sound while every op sees past minSeq (DocClients)
        if ref < clients.min_seq:
            raise MergeTreeError(MTE_E_INVALID_ARG, f"referenceSequenceNumber {ref} < minSeq {clients.min_seq}")
        recs = []
        if msg.get("type", "op") == "op":
            if sender == clients.observer:
                # our own op, sequenced: ackPendingSegment (client.ts:925-928)
                if not clients.local:
                    raise MergeTreeError(MTE_E_UNSUPPORTED, "ack of a local op in an observer document")
                if not clients.pending:
                    raise MergeTreeError(MTE_E_STATE, "ack without a pending local op")
                lo, hi = clients.pending[0]
                # the engine clears pending property keys up to hi (acks in
                # localSeq order, the runtime regenerating every pending op in
                # order); after a partial regeneration an earlier annotate can
                # still be pending here, whose keys that would clear
                if any(plo < lo and OP_ANNOTATE in pt
                       for (plo, _), pt in zip(clients.pending[1:], clients.pending_types[1:])):
                    raise MergeTreeError(MTE_E_UNSUPPORTED, "ack out of localSeq order past a pending annotate "
                                         "(regenerate every pending op, in order)")
                clients.pending.pop(0)
                types = clients.pending_types.pop(0)
                mask = 0
                for ls in range(lo, hi + 1):
                    if ls in clients.ann_slot:
                        mask |= 1 << clients.ann_slot.pop(ls)
                    elif types[ls - lo] == OP_ANNOTATE:
                        clients.untracked_acks += 1
                    # an annotate acked under a later pending one on the same key:
                    # the engine keeps the value from before the first pending
                    # annotate, not this one's, so the later one's rollback
                    # could not put this value back
                    keys = clients.ann_props.pop(ls, {})
                    for ls2, kv in clients.ann_props.items():
                        if ls2 > hi and keys.keys() & kv.keys():
                            clients.no_rollback.add(ls2)
                    clients.no_rollback.discard(ls)
                regen = lo in clients.regenerated
                clients.regenerated.discard(lo)
                flags, stamp = F_REGENERATED if regen else 0, NO_PROPS
                comb = clients.ann_comb.pop(hi, None)
                if comb is not None and comb[1].get("name") == "consensus":
                    # updateConsensusProperty: the marker's consensus value takes the seq
                    stamp = self.props.add_combining(comb[0], comb[1], seq)
                    flags |= F_COMBINE
                for ls in range(lo, hi):
                    clients.ann_comb.pop(ls, None)
                recs.append((OP_ACK, flags, lo, hi, mask, stamp))
            else:
                self._comb = (clients.local or clients.tree, seq)
                try:
                    self._op_records(msg.get("contents"), recs)
                finally:
                    self._comb = None
        # the slot is taken only once the message has validated
        short = clients.short(sender, seq)
        if short >= clients.max_clients:
            hint = "" if clients.max_clients == MTE_MAX_CLIENTS_TREE else \
                f" (a document flagged MTE_DOC_TREE takes {MTE_MAX_CLIENTS_TREE})"
            raise MergeTreeError(MTE_E_CLIENT_RANGE, f"client {sender!r}: more than {clients.max_clients} "
                                 f"clients inside the collab window{hint}")
        if not recs:
            recs.append((OP_NOOP, 0, 0, 0, 0, NO_PROPS))
        out = self.ops[doc]
        last = len(recs) - 1
        for i, (t, flags, p1, p2, a, b) in enumerate(recs):
            if t == OP_RELPOS:  # seq / ref_seq carry the offsets
                out.append((b[0], b[1], 0, t, short, flags, p1, p2, a, 0))
                continue
            if i == last:
                flags |= F_MSG_END
            out.append((seq, ref, msn, t, short, flags, p1, p2, a, b))
        clients.advance(msn)

    def add_local(self, doc: int, clients: DocClients, op: dict):
        """A local op of the document's own client (insertSegmentLocal /
        removeRangeLocal / annotateRangeLocal, client.ts:131-229): one MTE_F_LOCAL
        record per (GROUP member) op, each with the next localSeq
        (mergeTree.ts:1915, collabWindow.localSeq); the message's localSeqs join
        the pending list, acked in order by add_message."""
        if not clients.local:
            raise MergeTreeError(MTE_E_UNSUPPORTED, "local op in an observer document")
        recs = []
        # a local incr / consensus: its value map at seq UnassignedSequenceNumber
        # (-1), what annotateRange makes of every value (segmentPropertiesManager.ts:141)
        self._comb = (True, -1)
        try:
            self._op_records(op, recs)
        finally:
            self._comb = None
        if not recs:
            recs.append((OP_NOOP, 0, 0, 0, 0, NO_PROPS))
        if any(t != OP_RELPOS and f & F_REWRITE for t, f, *_ in recs):
            raise MergeTreeError(MTE_E_UNSUPPORTED, "local combiningOp rewrite")
        # a local consensus is annotateMarkerNotifyConsensus's (client.ts:137-158):
        # its ack stamps the marker's consensus value with the seq
        # (updateConsensusProperty, :646-650, 1083-1090), which needs the op's own
        # group slot and a message of that op alone; a consensus over a range
        # fails at its ack in the reference (relativePos1 undefined)
        cons = [i for i, r in enumerate(recs) if r[0] == OP_ANNOTATE and r[1] & F_COMBINE and
                self.props.comb_of[r[4]][1].get("name") == "consensus"]
        if cons:
            if len([r for r in recs if r[0] != OP_RELPOS]) != 1 or recs[0][0] != OP_RELPOS:
                raise MergeTreeError(MTE_E_UNSUPPORTED, "a local consensus annotate is a marker's "
                                     "(annotateMarkerNotifyConsensus), alone in its message")
            if len(clients.ann_slot) >= ANNOTATE_SLOTS:
                raise MergeTreeError(MTE_E_UNSUPPORTED, f"a local consensus annotate with {ANNOTATE_SLOTS} "
                                     "annotates pending")
        first = clients.local_seq + 1
        n_ops = sum(1 for r in recs if r[0] != OP_RELPOS)
        if first + n_ops >= LOCAL_SEQ_BASE:
            raise MergeTreeError(MTE_E_INVALID_ARG, "localSeq overflow")
        out = self.ops[doc]
        i = 0
        for t, flags, p1, p2, a, b in recs:
            if t == OP_RELPOS:  # takes no localSeq
                out.append((b[0], b[1], 0, t, 0, flags, p1, p2, a, 0))
                continue
            if t == OP_ANNOTATE:
                used = set(clients.ann_slot.values())
                free = next((x for x in range(ANNOTATE_SLOTS) if x not in used), None)
                if free is not None:
                    clients.ann_slot[first + i] = free
                    b = free
                f0, cnt = self.props.sets[a]
                if flags & F_COMBINE:
                    # its keys (the map's headers); what it sets depends on each
                    # segment, so no rollback restates it (nor one past it)
                    comb = self.props.comb_of[a]
                    clients.ann_props[first + i] = {k: None for k, n in self.props.entries[f0:f0 + cnt]
                                                    if not k & COMBINE_PAIR}
                    clients.ann_comb[first + i] = comb
                    clients.no_rollback.add(first + i)
                else:
                    clients.ann_props[first + i] = dict(self.props.entries[f0:f0 + cnt])
            out.append((first + i, 0, 0, t, 0, flags | F_LOCAL, p1, p2, a, b))
            i += 1
        clients.local_seq += n_ops
        clients.pending.append((first, clients.local_seq))
        clients.pending_types.append(tuple(r[0] for r in recs if r[0] != OP_RELPOS))

    def add_rollback(self, doc: int, clients: DocClients):
        """Client.rollback of the latest pending local op (client.ts:396-398 ->
        MergeTree.rollback, mergeTree.ts:2005-2083): one MTE_OP_ROLLBACK record
        per record of that op, last first.  An annotate's carries its group slot
        and is followed by its MTE_OP_RBKEY records (include/mte.h): per key it
        set, the older pending annotates that set the key, latest first, then
        the base entry.  MTE_E_UNSUPPORTED for an annotate the engine cannot
        restate: untracked (no group slot), an older untracked annotate on one
        of its keys, or an older annotate on one of its keys acked meanwhile."""
        if not clients.local or not clients.pending:
            raise MergeTreeError(MTE_E_STATE, "rollback without a pending local op")
        types = clients.pending_types[-1]
        lo, hi = clients.pending[-1]
        aux = {}
        for ls in range(hi, lo - 1, -1):
            if types[ls - lo] != OP_ANNOTATE:
                continue
            if ls not in clients.ann_slot or ls in clients.no_rollback:
                raise MergeTreeError(MTE_E_UNSUPPORTED, "rollback of an annotate the engine does not track")
            # a regenerated message moves behind newer ones; rolling it back under a
            # newer pending annotate of the same key leaves that key pending in the
            # reference (its count drops by one), which the engine does not restate
            if any(x > ls and x not in range(lo, hi + 1) and kv.keys() & clients.ann_props[ls].keys()
                   for x, kv in clients.ann_props.items()):
                raise MergeTreeError(MTE_E_UNSUPPORTED, "rollback under a newer pending annotate of the same key")
            recs = []
            for k, _ in clients.ann_props[ls].items():
                older = sorted((x for x, kv in clients.ann_props.items() if x < ls and k in kv), reverse=True)
                if any(x not in clients.ann_slot for x in older):
                    raise MergeTreeError(MTE_E_UNSUPPORTED, "rollback past an untracked pending annotate")
                if any(x in clients.ann_comb for x in older):
                    raise MergeTreeError(MTE_E_UNSUPPORTED, "rollback past a pending local incr / consensus")
                for x in older:
                    recs.append((x, 0, 0, OP_RBKEY, 0, F_LOCAL, k, clients.ann_slot[x], clients.ann_props[x][k],
                                 NO_PROPS))
                recs.append((0, 0, 0, OP_RBKEY, 0, F_LOCAL, k, ANNOTATE_SLOTS, 0, NO_PROPS))
            aux[ls] = recs
        clients.regenerated.discard(lo)
        clients.pending.pop()
        clients.pending_types.pop()
        out = self.ops[doc]
        for ls in range(hi, lo - 1, -1):
            t = types[ls - lo]
            if t == OP_ANNOTATE:
                out.append((ls, 0, 0, OP_ROLLBACK, 0, F_LOCAL, t, len(aux[ls]), clients.ann_slot.pop(ls), NO_PROPS))
                out.extend(aux[ls])
                del clients.ann_props[ls]
                clients.ann_comb.pop(ls, None)
            elif t != OP_NOOP:
                out.append((ls, 0, 0, OP_ROLLBACK, 0, F_LOCAL, t, 0, 0, NO_PROPS))

    def add_regen(self, doc: int, clients: DocClients):
        """Client.regeneratePendingOp of the oldest pending local message
        (client.ts:972-1002): one MTE_OP_REGEN record per record of it; the
        message moves to the end of the pending list (its groups are re-queued
        under the same localSeqs, resetPendingDeltaToOps :851-855).  Returns
        [(record index in the doc's part of the batch, localSeq, type)]; the
        engine reports the regenerated ops as MTE_DELTA_REGEN delta records of
        those indices (regen_ops turns them into ops)."""
        if not clients.local or not clients.pending:
            raise MergeTreeError(MTE_E_STATE, "regenerate without a pending local op")
        lo, hi = clients.pending[0]
        types = clients.pending_types[0]
        out = self.ops[doc]
        idx = []
        for ls in range(lo, hi + 1):
            t = types[ls - lo]
            if t == OP_NOOP:
                continue
            slot = 0
            if t == OP_ANNOTATE:
                if ls not in clients.ann_slot:
                    raise MergeTreeError(MTE_E_UNSUPPORTED, "regenerate an untracked annotate "
                                         f"(more than {ANNOTATE_SLOTS} pending)")
                slot = clients.ann_slot[ls]
            idx.append((len(out), ls, t))
            out.append((ls, 0, 0, OP_REGEN, 0, F_LOCAL, t, 0, slot, NO_PROPS))
        clients.regenerated.add(lo)
        clients.pending.append(clients.pending.pop(0))
        clients.pending_types.append(clients.pending_types.pop(0))
        return idx

    def add_ref(self, doc: int, clients: DocClients, pos: int, ref_type: int = REF_SLIDE_ON_REMOVE) -> int:
        """Client.createLocalReferencePosition on the segment and offset that
        getContainingSegment(pos) finds in the local view (client.ts:360-364,
        1107-1110; mergeTree.ts:872-885, 2124-2143): an MTE_OP_REF record in an
        MTE_DOC_REFS document.  A Transient one is its segment and offset, never
        moved or slid (localReference.ts:263).  Returns the reference's slot
        (mte_read_refs)."""
        if not clients.local:
            raise MergeTreeError(MTE_E_UNSUPPORTED, "local reference in an observer document")
        ref_type = _check_i32(ref_type, "refType")
        if ref_type < 0 or (ref_type & REF_TRANSIENT and ref_type & (REF_SLIDE_ON_REMOVE | REF_STAY_ON_REMOVE)):
            raise MergeTreeError(MTE_E_INVALID_ARG, "Transient with SlideOnRemove or StayOnRemove "
                                 "(localReference.ts:27-38)")
        if ref_type & REF_SLIDE_ON_REMOVE and ref_type & REF_STAY_ON_REMOVE:
            raise MergeTreeError(MTE_E_INVALID_ARG, "SlideOnRemove and StayOnRemove together")
        slot = _ref_slot(clients)
        self.ops[doc].append((0, 0, 0, OP_REF, 0, F_LOCAL, _check_i32(pos, "pos"), slot, ref_type, 0))
        return slot

    def add_rebase(self, doc: int, clients: DocClients, pos: int, seq_from: int, local_seq: int):
        """Client.rebasePosition(pos, seq_from, local_seq) (client.ts:755-786)
        for a pending interval op's reconnection (rebaseLocalInterval,
        intervalCollection.ts:1735-1803): an MTE_OP_REF record with b = 4,
        answered by one MTE_DELTA_REBASE event (the position, -1 detached)."""
        if not clients.local:
            raise MergeTreeError(MTE_E_UNSUPPORTED, "rebase in an observer document")
        if not 0 <= local_seq <= clients.local_seq:
            raise MergeTreeError(MTE_E_INVALID_ARG, f"localSeq {local_seq} > the client's {clients.local_seq}")
        self.ops[doc].append((0, _check_i32(seq_from, "seq"), 0, OP_REF, 0, F_LOCAL, _check_i32(pos, "pos"), 0,
                              local_seq, 4))

    def add_ref_rebase(self, doc: int, clients: DocClients, slot: int, local_seq: int):
        """rebaseLocalInterval's slide of a pending interval end
        (intervalCollection.ts:1782-1799): the reference in slot moves to its
        slide target's position in the view at local_seq if its segment is
        removed and acked (MTE_OP_REF b = 5; one MTE_DELTA_REBASE event, -1 when
        it stays)."""
        if not 0 <= slot < clients.ref_next or slot in clients.ref_free:
            raise MergeTreeError(MTE_E_INVALID_ARG, f"no local reference in slot {slot}")
        if not 0 <= local_seq <= clients.local_seq:
            raise MergeTreeError(MTE_E_INVALID_ARG, f"localSeq {local_seq} > the client's {clients.local_seq}")
        self.ops[doc].append((0, 0, 0, OP_REF, 0, F_LOCAL, 0, slot, local_seq, 5))

    def remove_ref(self, doc: int, clients: DocClients, slot: int):
        """removeLocalReferencePosition (mergeTree.ts:2113-2123)."""
        if not 0 <= slot < clients.ref_next or slot in clients.ref_free:
            raise MergeTreeError(MTE_E_INVALID_ARG, f"no local reference in slot {slot}")
        clients.ref_free.append(slot)
        self.ops[doc].append((0, 0, 0, OP_REF, 0, F_LOCAL, -1, slot, 0, 1))

    def _op_records(self, op, recs):
        if not isinstance(op, dict):
            raise MergeTreeError(MTE_E_INVALID_ARG, "op contents must be an object")
        t = op.get("type")
        if t == GROUP:
            for member in op.get("ops", []):
                self._op_records(member, recs)
            return
        rel = self._relpos(op, t)
        if t in (REMOVE, ANNOTATE) and "pos2" not in op and not (rel and rel[1] & RP_POS2):
            raise MergeTreeError(MTE_E_UNSUPPORTED, "range op without pos2")
        if rel and (t != INSERT or op.get("seg") is not None):
            recs.append(rel)
        p1 = op.get("pos1", 0 if (t == INSERT or (rel and rel[1] & RP_POS1)) else None)
        p2 = op.get("pos2", 0)
        if p1 is None:
            raise MergeTreeError(MTE_E_UNSUPPORTED, "range op without pos1")
        if t == INSERT:
            seg = op.get("seg")
            if seg is None:  # applyInsertOp returns false: no segment
                recs.append((OP_NOOP, 0, 0, 0, 0, NO_PROPS))
                return
            pos = _check_i32(p1, "pos1")
            if isinstance(seg, str):
                off, n = self._text(seg)
                recs.append((OP_INSERT, 0, pos, n, off, NO_PROPS))
            elif isinstance(seg, dict) and "text" in seg:
                off, n = self._text(seg["text"])
                recs.append((OP_INSERT, 0, pos, n, off, self.props.add(seg.get("props"))))
            elif isinstance(seg, dict) and "marker" in seg:
                ref_type = _check_i32(seg["marker"].get("refType", 0), "refType")
                # one reserved text unit names the marker in MTE_DOC_REFS documents
                off, _ = self._text("\ufffc")
                recs.append((OP_INSERT, F_MARKER, pos, ref_type, off, self.props.add(seg.get("props"))))
            else:
                raise MergeTreeError(MTE_E_INVALID_ARG, f"Unrecognized IJSONSegment type: {seg!r}")
        elif t == REMOVE:
            recs.append((OP_REMOVE, 0, _check_i32(p1, "pos1"), _check_i32(p2, "pos2"),
                         0, NO_PROPS))
        elif t == ANNOTATE:
            comb = op.get("combiningOp")
            flags = 0
            if comb is not None and comb.get("name") in ("incr", "consensus"):
                ctx = getattr(self, "_comb", None)
                if ctx is None:
                    raise MergeTreeError(MTE_E_UNSUPPORTED, f"local combiningOp {comb.get('name')!r}")
                if not ctx[0]:
                    raise MergeTreeError(MTE_E_UNSUPPORTED, f"combiningOp {comb.get('name')!r} outside a "
                                         "local-client or tree document (the HBM tree pass)")
                if comb.get("name") == "consensus" and "defaultValue" in comb:
                    raise MergeTreeError(MTE_E_UNSUPPORTED, "consensus with a defaultValue")
                ps = self.props.add_combining(op.get("props", {}), comb, ctx[1])
                recs.append((OP_ANNOTATE, F_COMBINE, _check_i32(p1, "pos1"), _check_i32(p2, "pos2"), ps, NO_PROPS))
                return
            if comb is not None:
                if comb.get("name") != "rewrite":
                    raise MergeTreeError(MTE_E_UNSUPPORTED, f"combiningOp {comb.get('name')!r}")
                flags = F_REWRITE
            ps = self.props.add(op.get("props", {}))
            recs.append((OP_ANNOTATE, flags, _check_i32(p1, "pos1"), _check_i32(p2, "pos2"), ps, NO_PROPS))
        else:
            raise MergeTreeError(MTE_E_INVALID_ARG, f"unknown op type {t!r}")

    def _relpos(self, op, t):
        """getValidOpRange (client.ts:541-560): a position given as relativePos
        (no pos1 / pos2) -> an MTE_OP_RELPOS record for the engine to resolve
        (posFromRelativePos, mergeTree.ts:1369-1392), or None."""
        flags, vids, offs = 0, [0, 0], [0, 0]
        for i, (pk, rk, pf, bf) in enumerate((("pos1", "relativePos1", RP_POS1, RP_BEFORE1),
                                               ("pos2", "relativePos2", RP_POS2, RP_BEFORE2))):
            rp = op.get(rk)
            if pk in op or rp is None or (i == 1 and t == INSERT):
                continue
            if not isinstance(rp, dict):
                raise MergeTreeError(MTE_E_INVALID_ARG, f"{rk} must be an object")
            flags |= pf
            if rp.get("before"):
                flags |= bf
            if rp.get("offset") is not None:
                offs[i] = _check_i32(rp["offset"], f"{rk}.offset")
            mid = rp.get("id")
            # an id no marker was ever given cannot match (value 0)
            vids[i] = self.interner.values.get(canonical_json(mid), 0) if mid else 0
        if not flags:
            return None
        key = self.interner.keys.get(MARKER_ID_KEY, NO_PROPS)
        return (OP_RELPOS, flags, vids[0], vids[1], key, (offs[0], offs[1]))

    def build(self):
        """-> dict of numpy arrays forming one mte_batch."""
        counts = np.array([len(o) for o in self.ops], dtype=np.uint64)
        offsets = np.zeros(self.n_docs + 1, dtype=np.uint64)
        np.cumsum(counts, out=offsets[1:])
        flat = [r for o in self.ops for r in o]
        ops = np.array(flat, dtype=OP_DTYPE) if flat else np.zeros(0, OP_DTYPE)
        text = np.concatenate(self.text) if self.text else np.zeros(0, dtype="<u2")
        ps, pe = self.props.arrays()
        return {"op_offsets": offsets, "ops": ops, "text": text.astype("<u2"),
                "propsets": ps, "props": pe}


def _members(op):
    """The merge-tree ops of a message's contents, GROUP flattened (one localSeq each)."""
    if isinstance(op, dict) and op.get("type") == GROUP:
        return [m for x in op.get("ops", []) for m in _members(x)]
    return [op]


def regen_ops(op, idx, deltas):
    """The regenerated op of Client.regeneratePendingOp (client.ts:972-1002,
    resetPendingDeltaToOps :788-860) from the engine's MTE_DELTA_REGEN records.

    op: the pending message's original contents; idx: add_regen's result;
    deltas: the doc's delta records (DELTA_DTYPE) of that batch.  One op per
    segment of each member's group, in document order: an insert re-sends the
    segment's part of the original text (with the original seg.props, if any,
    :829-832), a remove / annotate its range.  Returns one op, or a GROUP."""
    from .abi import DELTA_REGEN
    members = [m for m in _members(op) if not (m.get("type") == INSERT and m.get("seg") is None)]
    by_rec = {}
    for dl in deltas:
        if int(dl["kind"]) & DELTA_REGEN:
            by_rec.setdefault(int(dl["op"]), []).append(dl)
    out = []
    for (k, _ls, t), m in zip(idx, [m for m in members if m.get("type") in (INSERT, REMOVE, ANNOTATE)]):
        recs = by_rec.get(k, [])
        if t == INSERT:
            seg = m["seg"]
            base = min((int(r["removed"]) for r in recs), default=0)
            for r in recs:
                p, n = int(r["pos"]), int(r["len"])
                if isinstance(seg, str):
                    u = utf16_units(seg)
                    o = int(r["removed"]) - base
                    s = u[o:o + n].tobytes().decode("utf-16-le")
                    out.append({"pos1": p, "seg": s, "type": INSERT})
                elif "text" in seg:
                    u = utf16_units(seg["text"])
                    o = int(r["removed"]) - base
                    s = {"text": u[o:o + n].tobytes().decode("utf-16-le")}
                    if seg.get("props") is not None:
                        s["props"] = seg["props"]
                    out.append({"pos1": p, "seg": s, "type": INSERT})
                else:
                    out.append({"pos1": p, "seg": seg, "type": INSERT})
        elif t == REMOVE:
            out += [{"pos1": int(r["pos"]), "pos2": int(r["pos"]) + int(r["len"]), "type": REMOVE} for r in recs]
        else:
            for r in recs:
                a = {"pos1": int(r["pos"]), "pos2": int(r["pos"]) + int(r["len"]), "props": m.get("props", {}),
                     "type": ANNOTATE}
                if m.get("combiningOp") is not None:
                    a["combiningOp"] = m["combiningOp"]
                out.append(a)
    return out[0] if len(out) == 1 else {"ops": out, "type": GROUP}

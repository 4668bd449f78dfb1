// Type declarations of the MI355X batched sequence-merge engine's host layer
// (index.js).  The surface mirrors @fluidframework/merge-tree's Client /
// MergeTree for the remote-op path (packages/dds/merge-tree/src/client.ts,
// mergeTree.ts); see index.js for the reference file:line of each member.

export type PropertySet = { [key: string]: any };

export interface ICombiningOp {
  name: string;
  defaultValue?: any;
}

/** IJSONSegment as carried by insert ops (ops.ts, textSegment.ts:40-48, mergeTreeNodes.ts:602-609). */
export type IJSONSegment =
  | string
  | { text: string; props?: PropertySet }
  | { marker: { refType?: number }; props?: PropertySet };

export interface IMergeTreeOp {
  type: 0 | 1 | 2 | 3;
  pos1?: number;
  pos2?: number;
  seg?: IJSONSegment;
  props?: PropertySet;
  combiningOp?: ICombiningOp;
  ops?: IMergeTreeOp[];
}

/** The fields of ISequencedDocumentMessage the path reads (protocol.ts:212). */
export interface ISequencedDocumentMessage {
  clientId: string | null;
  sequenceNumber: number;
  referenceSequenceNumber: number;
  minimumSequenceNumber: number;
  type: string;
  contents: IMergeTreeOp | any;
}

export interface EngineOptions {
  device?: number;
  nKeys?: number;
  segCapacity?: number;
  /** local reference slots per document (mte_set_ref_capacity, default 1024); a
   *  reference past it throws for its document (MergeTreeError code -4) */
  refCapacity?: number;
}

/** IJSONSegmentWithMergeInfo (snapshotChunks.ts:48-78): one segment of a summary body. */
export interface SegmentWithMergeInfo {
  json: string | { text: string; props?: PropertySet } | { marker: { refType: number }; props?: PropertySet };
  client?: string;
  seq?: number;
  removedSeq?: number;
  removedClient?: string;
  removedClientIds?: string[];
}

export interface ClientOptions {
  observerId?: string;
  /** This client sends ops of its own (MTE_DOC_LOCAL_CLIENT; needs newLengthCalc):
   *  observerId / longClientId name it, its sequenced messages are acks. */
  localClient?: boolean;
  longClientId?: string;
  /** Record delta events (MTE_DOC_EVENTS; needs newLengthCalc): BatchClient.on("sequenceDelta"). */
  events?: boolean;
  /** Hold local references (MTE_DOC_REFS; needs localClient): createLocalReferencePosition. */
  refs?: boolean;
  /** mergeTreeMaintenanceCallback records -> BatchClient.on("maintenance") (needs localClient, events). */
  maintenanceEvents?: boolean;
  /** MTE_DOC_TREE: replay on the tree pass (the reference's segmentation; segment-exact sequenceDelta ranges;
   *  up to 63 senders inside one collab window, 31 on the flat passes). */
  tree?: boolean;
  newLengthCalc?: boolean;
  props?: PropertySet;
  minSeq?: number;
  currentSeq?: number;
  /** Declare the document's stream round-synchronous (MTE_DOC_ROUND_SYNC): a
   *  legacy length-calc document then replays on the flat passes; a batch
   *  breaking the declaration stops it with code -9. */
  roundSync?: boolean;
  /** Load a summary body instead of initialText (SnapshotLoader.loadBody). */
  segments?: SegmentWithMergeInfo[];
  /** Load a legacy summary (SnapshotLegacy blobs) and queue its catch-up ops. */
  legacy?: LegacySummary;
  /** Load the blobs of either summary format (summarizeV1 / summarizeLegacy). */
  summary?: LegacySummary | V1Summary;
}

/** MergeTreeChunkV1 (snapshotChunks.ts:47-55) as SnapshotV1.emit writes it. */
export interface V1Chunk {
  version: "1";
  segmentCount: number;
  length: number;
  segments: any[];
  startIndex: number;
  headerMetadata?: { minSequenceNumber: number; sequenceNumber: number; orderedChunkMetadata: { id: string }[];
    totalLength: number; totalSegmentCount: number };
}

/** "header" plus "body_0", "body_1", ... */
export interface V1Summary {
  header: V1Chunk;
  [bodyId: string]: V1Chunk;
}

/** MergeTreeChunkLegacy (snapshotChunks.ts:22-34) as SnapshotLegacy.emit writes it. */
export interface LegacyChunk {
  chunkStartSegmentIndex: number;
  chunkSegmentCount: number;
  chunkLengthChars: number;
  totalLengthChars: number;
  totalSegmentCount: number;
  chunkSequenceNumber: number;
  segmentTexts: any[];
  headerMetadata?: { orderedChunkMetadata: { id: string }[]; sequenceNumber: number;
    minSequenceNumber?: number; totalLength: number; totalSegmentCount: number };
}

export interface LegacySummary {
  header: LegacyChunk;
  body?: LegacyChunk;
  catchupOps?: ISequencedDocumentMessage[];
}

export class MergeTreeError extends Error {
  code: number;
  assertCode?: number;
}

export interface EngineStats {
  opsApplied: number;
  segsScanned: number;
  chunkScanned?: number;
  /** the round phases' bytes read and written in the last run (mte_stats.round_bytes) */
  roundBytes?: number;
  segsWritten: number;
  propWrites: number;
  unitsInserted: number;
  maxSegs: number;
  kernelMs: number;
  algoBytes: number;
}

export class MergeTreeEngine {
  constructor(options?: EngineOptions);
  readonly nKeys: number;
  createClient(initialText?: string, options?: ClientOptions): BatchClient;
  start(): void;
  /** Launch the replay of every queued message (returns before it ends). */
  flush(): void;
  /** Wait for the launched replay (every read-out does). */
  sync(): void;
  /** Delta-event records per op record of {events: true} documents (mte_set_event_capacity). */
  setEventCapacity(perOp: number): void;
  digests(): BigUint64Array;
  statuses(): Int32Array;
  stats(): EngineStats;
  close(): void;
  /** Node level (one process per GPU, RCCL over xGMI, mte_comm_*). */
  commUniqueId(): Uint8Array;
  joinNode(world: number, rank: number, id: Uint8Array): void;
  shareNode(other: MergeTreeEngine): void;
  nodeBarrier(): void;
  nodeAllreduce(value: number, op?: "sum" | "max"): number;
  gatherDigests(docsPerRank: number): BigUint64Array;
  leaveNode(): void;
  /** Documents -> ranks by expected work (LPT). */
  static shardByWork(work: number[], world: number): number[];
}

export interface BatchMergeTree {
  insertSegments(pos: number, segments: Array<IJSONSegment | { toJSONObject(): IJSONSegment }>,
    refSeq: number, clientId: number, seq: number): void;
  markRangeRemoved(start: number, end: number, refSeq: number, clientId: number, seq: number): void;
  annotateRange(start: number, end: number, props: PropertySet, combiningOp: ICombiningOp | undefined,
    refSeq: number, clientId: number, seq: number): void;
}

export interface VisibleSegment {
  kind: "text" | "marker";
  text?: string;
  refType?: number;
  length: number;
  props?: PropertySet;
}

export interface SequenceDeltaRange {
  position: number;   // Client.getPosition of the segment in this client's view after the op
  length: number;     // cachedLength
  removed: boolean;   // removed in this client's view
  segment?: unknown;  // an insert's segment spec
}
export interface SequenceDeltaEvent {
  deltaOperation: number;  // MergeTreeDeltaType
  operation: "insert" | "remove" | "annotate";
  isLocal: boolean;
  message?: ISequencedDocumentMessage;
  ranges: SequenceDeltaRange[];
  first: SequenceDeltaRange;
  last: SequenceDeltaRange;
}

/** SequenceMaintenanceEvent (sequenceDeltaEvent.ts:128-136): one mergeTreeMaintenanceCallback. */
export interface SequenceMaintenanceEvent {
  deltaOperation: number;  // MergeTreeMaintenanceType: APPEND -1, SPLIT -2, UNLINK -3, ACKNOWLEDGED -4
  operation: "append" | "split" | "unlink" | "acknowledged";
  opArgs: { op: any; sequencedMessage?: ISequencedDocumentMessage } | undefined;
  clientId: string;
  /** position in the client's view once the message is applied (-1: unlinked), length at the callback */
  ranges: { operation: number; position: number; length: number; propertyDeltas: PropertySet; segment: undefined }[];
  first: { operation: number; position: number; length: number };
  last: { operation: number; position: number; length: number };
}

/** ReferenceType flags (ops.ts): Simple 0, SlideOnRemove 0x40, StayOnRemove 0x80, Transient 0x100. */
export class LocalReferencePosition {
  readonly refType: number;
  properties?: PropertySet;
  addProperties(newProps: PropertySet): void;
  getProperties(): PropertySet | undefined;
}

/** getContainingSegment's snapshot of a visible segment. */
export interface SegmentSnapshot {
  start: number;
  length: number;
  kind: number;
}

/** IntervalType (intervalCollection.ts:48-66) and ReferenceType (merge-tree ops.ts) flags. */
export const IntervalType: { Simple: 0; Nest: 1; SlideOnRemove: 2; Transient: 4 };
export const RefType: { Simple: 0; Tile: 1; NestBegin: 2; NestEnd: 4; RangeBegin: 16; RangeEnd: 32;
  SlideOnRemove: 64; StayOnRemove: 128; Transient: 256 };

/** SequenceInterval (intervalCollection.ts:387-619): its ends are engine references. */
export class SequenceInterval {
  start: LocalReferencePosition;
  end: LocalReferencePosition;
  intervalType: number;
  properties: PropertySet;
  getIntervalId(): string;
  /** [start, end] in the client's view (-1: slid off the string). */
  positions(): [number, number];
  serialize(): { start: number; end: number; intervalType: number; sequenceNumber: number; properties: PropertySet };
}

/** IntervalCollection (intervalCollection.ts:1309-2102) over a {localClient, refs} BatchClient. */
export class IntervalCollection implements Iterable<SequenceInterval> {
  readonly label: string;
  add(start: number, end: number, intervalType: number, props?: PropertySet): SequenceInterval;
  change(id: string, start?: number, end?: number): SequenceInterval | undefined;
  changeProperties(id: string, props: PropertySet): void;
  removeIntervalById(id: string): SequenceInterval | undefined;
  getIntervalById(id: string): SequenceInterval | undefined;
  /** A sequenced interval op (makeOpsMap): ackAdd / ackChange / ackDelete. */
  process(opName: "add" | "change" | "delete", value: any, local: boolean, op: ISequencedDocumentMessage): void;
  findOverlappingIntervals(startPosition: number, endPosition: number): SequenceInterval[];
  previousInterval(pos: number): SequenceInterval | undefined;
  nextInterval(pos: number): SequenceInterval | undefined;
  CreateForwardIteratorWithStartPosition(startPosition: number): Iterator<SequenceInterval>;
  CreateBackwardIteratorWithStartPosition(startPosition: number): Iterator<SequenceInterval>;
  CreateForwardIteratorWithEndPosition(endPosition: number): Iterator<SequenceInterval>;
  CreateBackwardIteratorWithEndPosition(endPosition: number): Iterator<SequenceInterval>;
  /** addInterval / deleteInterval / changeInterval / propertyChanged (intervalCollection.ts:1257-1300). */
  on(event: "addInterval" | "deleteInterval" | "changeInterval" | "propertyChanged", listener: (...args: any[]) => void): this;
  off(event: string, listener: (...args: any[]) => void): this;
  /** ISerializedIntervalCollectionV2 (:1968-1977); loads back through getIntervalCollection(label, emitter, serialized). */
  serializeInternal(): { label: string; intervals: any[]; version: 2 };
  /** The value type's rebase of a pending op for re-sending (makeOpsMap :1163-1172): deletes unchanged,
   *  adds / changes through rebaseLocalInterval; undefined: send the op empty. meta: the emitter's 4th argument. */
  rebaseOp(opName: "add" | "change" | "delete", value: any, meta: { localSeq: number }): any;
  /** rebaseLocalInterval (:1735-1803); needs an {events: true} document. */
  rebaseLocalInterval(opName: "add" | "change", value: any, localSeq: number): any;
  [Symbol.iterator](): Iterator<SequenceInterval>;
}

export class BatchClient {
  readonly mergeTree: BatchMergeTree;
  /** SharedString.getIntervalCollection; emitter.emit(opName, undefined, value) receives the ops to send. */
  getIntervalCollection(label: string, emitter?: { emit(opName: string, prev: undefined, value: any, meta: any): void }):
    IntervalCollection;
  /** A sequenced {key: label, type: "act", value: {opName, value}} interval message (applyMsg routes them too). */
  applyIntervalMsg(msg: ISequencedDocumentMessage): void;
  // local references ({localClient: true, refs: true} documents)
  getContainingSegment(pos: number): { segment: SegmentSnapshot | undefined; offset: number | undefined };
  createLocalReferencePosition(segment: SegmentSnapshot | number, offset: number | undefined, refType: number,
    properties?: PropertySet): LocalReferencePosition;
  removeLocalReferencePosition(lref: LocalReferencePosition): LocalReferencePosition | undefined;
  /** -1 (DetachedReferencePosition) once detached or removed. */
  localReferencePositionToPosition(lref: LocalReferencePosition): number;
  readonly longClientId: string;
  /** A remote message, or (localClient documents) the sequenced message of an own op: its ack. */
  applyMsg(msg: ISequencedDocumentMessage, local?: boolean): void;
  // local ops ({localClient: true, newLengthCalc: true} documents); each returns the op to send
  insertTextLocal(pos: number, text: string, props?: PropertySet): IMergeTreeOp;
  insertMarkerLocal(pos: number, refType: number, props?: PropertySet): IMergeTreeOp;
  insertSegmentLocal(pos: number, segment: unknown): IMergeTreeOp;
  removeRangeLocal(start: number, end: number): IMergeTreeOp;
  /** combiningOp rewrite, incr (and consensus, though the reference's ack then needs a marker's relative position). */
  annotateRangeLocal(start: number, end: number, props: PropertySet, combiningOp?: { name: string }): IMergeTreeOp;
  /** Client.annotateMarker: the marker by id (or an object with getId()); its position resolved by the engine. */
  annotateMarker(marker: string | { getId(): string }, props: PropertySet, combiningOp?: { name: string }):
    IMergeTreeOp | undefined;
  /** Client.annotateMarkerNotifyConsensus: a consensus annotate whose ack stamps the marker's value with the
   *  seq; consensusCallback(marker) once minSeq reaches that seq. */
  annotateMarkerNotifyConsensus(marker: string | { getId(): string }, props: PropertySet,
    consensusCallback: (marker: any) => void): IMergeTreeOp | undefined;
  /** A local op as its IMergeTreeDeltaOp JSON (relative positions included). */
  applyLocalOp(op: IMergeTreeOp): IMergeTreeOp;
  makeOpMessage(op: IMergeTreeOp, seq?: number, refSeq?: number, minSeq?: number): ISequencedDocumentMessage;
  getPendingCount(): number;
  /** Client.regeneratePendingOp for reconnection: the op re-sending the oldest
   *  pending op (resetOp as sent); needs {localClient: true, events: true}. */
  regeneratePendingOp(resetOp: IMergeTreeOp): IMergeTreeOp;
  /** Client.rollback of the latest pending local op (inserts, removes and annotates). */
  rollback(op?: IMergeTreeOp): void;
  /** SharedString "sequenceDelta" events ({events: true} documents), delivered at each flush in op order. */
  on(name: "sequenceDelta", listener: (event: SequenceDeltaEvent, client: BatchClient) => void): this;
  /** SharedString "maintenance" events ({maintenanceEvents: true} documents): SPLIT / APPEND / UNLINK /
   *  ACKNOWLEDGED callbacks (deltaOperation -2 / -1 / -3 / -4), ranges at the message's end. */
  on(name: "maintenance", listener: (event: SequenceMaintenanceEvent, client: BatchClient) => void): this;
  /** The catch-up stash of a legacy summary, ops rewritten to refSeq = seq - 1 (sequence.ts:688-725). */
  getMessagesSinceMSNChange(): ISequencedDocumentMessage[];
  getOrAddShortClientId(longId: string): number;
  getClientId(): number;
  getLongClientId(shortId: number): string | undefined;
  flush(): void;
  /** TestClient.getText(start?, end?): markers count one position, contribute no text. */
  getText(start?: number, end?: number): string;
  getLength(): number;
  getCurrentSeq(): number;
  getCollabWindow(): { clientId: number; currentSeq: number; minSeq: number; collaborating: boolean };
  getPropertiesAtPosition(pos: number): PropertySet | undefined;
  getSegments(): VisibleSegment[];
  /** Summary body (SnapshotV1.extractSegment rules) + the collab window to load it with. */
  summarize(): { segments: SegmentWithMergeInfo[]; minSeq: number; currentSeq: number };
  /** SnapshotV1.extractSync + emit (snapshotV1.ts:117-268): header + body_N chunks. */
  summarizeV1(chunkSize?: number): V1Summary;
  /** SnapshotLegacy.extractSync + emit (snapshotlegacy.ts:105-211). */
  summarizeLegacy(catchUpMsgs?: ISequencedDocumentMessage[], chunkSize?: number): LegacySummary;
}

// ref_stubs.js — the few values the erased reference merge-tree (oracle/ts_erase.py)
// imports from Fluid packages outside packages/dds/merge-tree (TEST INFRASTRUCTURE).
// Semantics follow the reference packages they stand in for:
//   assert(cond, msg)            common/lib/common-utils/src/assert.ts:15
//   Trace                        common/lib/common-utils/src/trace.ts:12-32
//   unreachableCase, bufferToString
//   UsageError / LoggingError    container-utils, telemetry-utils
//   MessageType.Operation = "op" protocol-definitions/src/protocol.ts:58
"use strict";

function assert(condition, message) {
  if (!condition) {
    const m = typeof message === "number" ? `0x${message.toString(16).padStart(3, "0")}` : message;
    throw new Error(m);
  }
}

class Trace {
  static start() {
    return new Trace(Date.now());
  }
  constructor(startTick) {
    this.startTick = startTick;
    this.lastTick = startTick;
  }
  trace() {
    const tick = Date.now();
    const event = { totalTimeElapsed: tick - this.startTick, duration: tick - this.lastTick, tick };
    this.lastTick = tick;
    return event;
  }
}

function unreachableCase(x, message = "Unreachable Case") {
  throw new Error(message);
}

function bufferToString(blob, encoding) {
  return Buffer.from(blob).toString(encoding);
}

class UsageError extends Error {}
class LoggingError extends Error {
  constructor(message, props) {
    super(message);
    Object.assign(this, props || {});
  }
}

const MessageType = {
  NoOp: "noop",
  ClientJoin: "join",
  ClientLeave: "leave",
  Propose: "propose",
  Reject: "reject",
  Summarize: "summarize",
  SummaryAck: "summaryAck",
  SummaryNack: "summaryNack",
  Operation: "op",
};

const AttachState = { Detached: "Detached", Attaching: "Attaching", Attached: "Attached" };

class ChildLogger {
  static create(logger) {
    return logger || { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };
  }
}

class SummaryTreeBuilder {
  constructor() {
    this.tree = {};
  }
  addBlob(key, content) {
    this.tree[key] = { type: 2, content };
  }
  addWithStats(key, value) {
    this.tree[key] = value.summary;
  }
  getSummaryTree() {
    return { summary: { type: 1, tree: this.tree }, stats: {} };
  }
}

module.exports = {
  assert,
  Trace,
  unreachableCase,
  bufferToString,
  UsageError,
  LoggingError,
  MessageType,
  AttachState,
  ChildLogger,
  SummaryTreeBuilder,
};

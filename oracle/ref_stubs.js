// ref_stubs.js — what the erased reference merge-tree (oracle/ts_erase.py) imports
// from Fluid packages that cannot be erased here (TEST INFRASTRUCTURE).  Every
// other imported value — assert, Trace, unreachableCase, bufferToString,
// MessageType, AttachState — is erased from the reference's own sources
// (ts_erase.py EXTERNAL).  What stays here carries none of the merge arithmetic:
//   ChildLogger                  telemetry-utils: a logger factory (no-op sink)
//   LoggingError / UsageError    telemetry-utils errorLogging.ts:360 / container-utils
//                                error.ts:77 — their module needs the third-party
//                                `uuid`, absent offline; raised only on failure
//                                paths (message + props kept)
//   SummaryTreeBuilder           runtime-utils summaryUtils.ts:128 — needs
//                                protocol-base; on no path the oracle runs
//   bufferToString               common-utils bufferNode.ts:58 (the same one-liner
//                                over Node's Buffer; that file's ambient class
//                                declaration defeats the eraser); summary load only
"use strict";

class ChildLogger {
  static create(logger) {
    return logger || { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };
  }
}

class LoggingError extends Error {
  constructor(message, props) {
    super(message);
    Object.assign(this, props || {});
  }
}
class UsageError extends LoggingError {}

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

const bufferToString = (blob, encoding) => Buffer.from(blob).toString(encoding);

module.exports = { ChildLogger, LoggingError, UsageError, SummaryTreeBuilder, bufferToString };

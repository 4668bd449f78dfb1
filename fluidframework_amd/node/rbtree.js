"use strict";
// The ordered map an IntervalCollection keeps its intervals' ends in
// (LocalIntervalCollection.endIntervalTree, intervalCollection.ts:728-757):
// merge-tree's RedBlackTree (collections/rbTree.ts), a left-leaning red-black
// tree (Sedgewick's 2-3 variant) whose behaviour the collection's
// previousInterval / nextInterval expose (floor / ceil, :897-913), so its rules
// are restated here, not an ordered list's:
//   * put(key, data, conflict): a key comparing equal to a node's replaces the
//     node's data and keeps the node's key unless conflict gives one
//     (rbTree.ts:249-300) -- intervals sharing an end share a node;
//   * remove(key): the node comparing equal to key goes, whatever interval it
//     holds, and only if contains(key) (rbTree.ts:323-372);
//   * the shape follows the same rotations and colour flips, so floor / ceil
//     walk the same nodes even when a node's key no longer compares as it did
//     when it was put (an end that moved without a remove / put).
// The comparison is the caller's, evaluated at the time of each call.

const RED = 0, BLACK = 1;

/** remove(key) walked off the tree: contains(key) found a node, but a node
 *  on the way no longer compares as it did when it was put (an end that moved
 *  without a remove / put), so the descent toward it left the tree. */
class KeyMovedError extends Error {}

class Node {
  constructor(key, data, color) {
    this.key = key;
    this.data = data;
    this.color = color;
    this.left = undefined;
    this.right = undefined;
  }
}

const isRed = (n) => n !== undefined && n.color === RED;

class RedBlackTree {
  constructor(compare) {
    this.compare = compare;
    this.root = undefined;
  }

  isEmpty() {
    return this.root === undefined;
  }

  _get(node, key) {
    while (node !== undefined) {
      const c = this.compare(key, node.key);
      if (c === 0) return node;
      node = c < 0 ? node.left : node.right;
    }
    return undefined;
  }

  contains(key) {
    return this._get(this.root, key) !== undefined;
  }

  put(key, data, conflict) {
    if (key === undefined) return;
    if (data === undefined) {
      this.remove(key);
      return;
    }
    this.root = this._put(this.root, key, data, conflict);
    this.root.color = BLACK;
  }

  _put(node, key, data, conflict) {
    if (node === undefined) return new Node(key, data, RED);
    const c = this.compare(key, node.key);
    if (c < 0) node.left = this._put(node.left, key, data, conflict);
    else if (c > 0) node.right = this._put(node.right, key, data, conflict);
    else if (conflict) {
      const kd = conflict(key, node.key, data, node.data);
      if (kd.key) node.key = kd.key;
      node.data = kd.data ? kd.data : data;
    } else {
      node.data = data;
    }
    if (isRed(node.right) && !isRed(node.left)) node = this._rotateLeft(node);
    if (isRed(node.left) && isRed(node.left.left)) node = this._rotateRight(node);
    if (isRed(node.left) && isRed(node.right)) this._flip(node);
    return node;
  }

  remove(key) {
    if (key === undefined || !this.contains(key)) return;
    if (!isRed(this.root.left) && !isRed(this.root.right)) this.root.color = RED;
    // the root keeps the colour the removal leaves it (rbTree.ts removeExisting
    // does not blacken it; the next put does)
    this.root = this._remove(this.root, key);
  }

  _remove(node, key) {
    if (this.compare(key, node.key) < 0) {
      if (node.left === undefined) throw new KeyMovedError("the removal left the tree");
      if (!isRed(node.left) && !isRed(node.left.left)) node = this._moveRedLeft(node);
      node.left = this._remove(node.left, key);
    } else {
      if (isRed(node.left)) node = this._rotateRight(node);
      if (this.compare(key, node.key) === 0 && node.right === undefined) return undefined;
      if (node.right === undefined) throw new KeyMovedError("the removal left the tree");
      if (!isRed(node.right) && !isRed(node.right.left)) node = this._moveRedRight(node);
      if (this.compare(key, node.key) === 0) {
        let m = node.right;
        while (m.left !== undefined) m = m.left;
        node.key = m.key;
        node.data = m.data;
        node.right = this._removeMin(node.right);
      } else {
        node.right = this._remove(node.right, key);
      }
    }
    return this._balance(node);
  }

  _removeMin(node) {
    if (node.left === undefined) return undefined;
    if (!isRed(node.left) && !isRed(node.left.left)) node = this._moveRedLeft(node);
    node.left = this._removeMin(node.left);
    return this._balance(node);
  }

  /** the largest node comparing <= key (rbTree.ts nodeFloor) */
  floor(key) {
    let node = this.root, best;
    while (node !== undefined) {
      const c = this.compare(key, node.key);
      if (c === 0) return node;
      if (c < 0) node = node.left;
      else {
        best = node;
        node = node.right;
      }
    }
    return best;
  }

  /** the smallest node comparing >= key (rbTree.ts nodeCeil) */
  ceil(key) {
    let node = this.root, best;
    while (node !== undefined) {
      const c = this.compare(key, node.key);
      if (c === 0) return node;
      if (c > 0) node = node.right;
      else {
        best = node;
        node = node.left;
      }
    }
    return best;
  }

  _rotateLeft(h) {
    const x = h.right;
    h.right = x.left;
    x.left = h;
    x.color = h.color;
    h.color = RED;
    return x;
  }

  _rotateRight(h) {
    const x = h.left;
    h.left = x.right;
    x.right = h;
    x.color = h.color;
    h.color = RED;
    return x;
  }

  _flip(h) {
    h.color = h.color === RED ? BLACK : RED;
    h.left.color = h.left.color === RED ? BLACK : RED;
    h.right.color = h.right.color === RED ? BLACK : RED;
  }

  _moveRedLeft(h) {
    this._flip(h);
    if (isRed(h.right.left)) {
      h.right = this._rotateRight(h.right);
      h = this._rotateLeft(h);
      this._flip(h);
    }
    return h;
  }

  _moveRedRight(h) {
    this._flip(h);
    if (isRed(h.left.left)) {
      h = this._rotateRight(h);
      this._flip(h);
    }
    return h;
  }

  _balance(h) {
    if (isRed(h.right)) h = this._rotateLeft(h);
    if (isRed(h.left) && isRed(h.left.left)) h = this._rotateRight(h);
    if (isRed(h.left) && isRed(h.right)) this._flip(h);
    return h;
  }
}

module.exports = { RedBlackTree, KeyMovedError };

// Synchronous TransformStream stand-in for Node 12 (no WHATWG streams there).
// Only what the reference bundle's CompressionStream/DecompressionStream use:
// transform/flush callbacks, a controller with enqueue(), writable.write/close
// and readable.pipeThrough().  Output chunks are collected for _drain().
class SyncTransformStream {
  constructor(tr) {
    this._out = [];
    this._sink = null;
    this._close = null;
    const ctrl = { enqueue: (x) => (this._sink ? this._sink(x) : this._out.push(x)) };
    if (tr.start) tr.start(ctrl);
    this.writable = {
      write: (c) => tr.transform(c, ctrl),
      close: () => { if (tr.flush) tr.flush(ctrl); if (this._close) this._close(); },
    };
    this.readable = {
      pipeThrough: (next) => {
        this._sink = (x) => next.writable.write(x);
        this._close = () => next.writable.close();
        return next.readable;
      },
      _drain: () => this._out.splice(0),
    };
  }
}
globalThis.TransformStream = SyncTransformStream;

"""The host -> device hand-off of the training batches.

The reference assembles each numpy batch in the training loop (or in a
torch.multiprocessing preloader, base.py:97-137) and the model copies it to
the device with synchronous, pageable np2var copies at the start of forward
(base.py:362-390, ctc.py:294-297), so the GPU idles while the host prepares
and copies.  Here a background thread runs one to ``depth`` batches ahead:

  1. the dataset assembles the padded, length-sorted batch and it is staged in
     pinned host memory (torch's caching host allocator), off the main thread;
  2. the features, the lengths and the blank-shifted flat label array (the
     CTC kernel's input, ctc.py:300 + _concatenate_labels :532-549, already in
     the batch's descending-length order, so no permutation) are copied to
     the device asynchronously on a dedicated copy stream;
  3. an event marks the copies; ``next()`` makes the compute stream wait on it
     (no host sync) and records the tensors on the compute stream.

``next()`` returns (batch, is_new_epoch): the host arrays of the reference's
batch dict plus 'xs' replaced by the device tensor and device int32 tensors
'x_lens_d', 'y_lens_d', 'labels_d' (+1 shifted, flat).  The models accept a
device 'xs' wherever the reference takes the numpy array.
"""
import queue
import threading

import numpy as np
import torch


class DeviceBatches(object):
    def __init__(self, dataset, device, depth=2):
        self.dataset = dataset
        self.device = torch.device(device)
        self.depth = max(1, int(depth))
        self.copy_stream = torch.cuda.Stream(device=self.device)
        self._q = queue.Queue(maxsize=self.depth)
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, daemon=True)
        self._thread.start()

    # ------------------------------------------------------------ producer
    def _stage(self, batch):
        xs = batch['xs']
        dev = self.device
        host = {}
        host['xs'] = torch.from_numpy(np.ascontiguousarray(xs)).pin_memory()
        yl = np.asarray(batch['y_lens'], np.int32)
        ys = np.asarray(batch['ys'])
        mask = np.arange(ys.shape[1])[None, :] < yl[:, None]
        host['labels'] = torch.from_numpy(np.ascontiguousarray(ys[mask] + 1, np.int32)).pin_memory()
        host['x_lens'] = torch.from_numpy(np.asarray(batch['x_lens'], np.int32)).pin_memory()
        host['y_lens'] = torch.from_numpy(yl).pin_memory()
        with torch.cuda.stream(self.copy_stream):
            out = {k: v.to(dev, non_blocking=True) for k, v in host.items()}
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
        return out, ev, host

    def _run(self):
        torch.cuda.set_device(self.device)
        try:
            while not self._stop.is_set():
                try:
                    batch, new_epoch = self.dataset.next()
                except StopIteration:
                    self._q.put(None)
                    return
                dev, ev, host = self._stage(batch)
                self._q.put((batch, new_epoch, dev, ev, host))
        except Exception as e:          # surfaced by next()
            self._q.put(e)

    # ------------------------------------------------------------ consumer
    def __iter__(self):
        return self

    def __next__(self):
        item = self._q.get()
        if item is None:
            raise StopIteration
        if isinstance(item, Exception):
            raise item
        batch, new_epoch, dev, ev, _host = item
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(ev)
        for t in dev.values():
            t.record_stream(cur)
        out = dict(batch)
        out['xs'] = dev['xs']
        out['x_lens_d'] = dev['x_lens']
        out['y_lens_d'] = dev['y_lens']
        out['labels_d'] = dev['labels']
        return out, new_epoch

    next = __next__

    def close(self):
        self._stop.set()
        try:
            while True:
                self._q.get_nowait()
        except queue.Empty:
            pass
        self._thread.join(timeout=5)

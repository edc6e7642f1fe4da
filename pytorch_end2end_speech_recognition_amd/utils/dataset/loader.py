"""Utterance dataset and padded, length-sorted mini-batch assembly: the
reference's DatasetBase / Base (utils/dataset/loader.py:29-157,
utils/dataset/base.py:76-201) with the corpus Dataset's filtering, sorting and
dynamic batch halving (examples/librispeech/s5/exp/dataset/load_dataset.py
:104-142), over the same CSV table (columns frame_num, input_path,
transcript).

Same contract: ``next(batch_size=None) -> (batch, is_new_epoch)`` with batch =
{'xs' f32 [B, T_max, F] zero-padded, 'ys' int32 [B, L_max] padded -1,
'x_lens' int32 [B], 'y_lens' int32 [B], 'input_names'}; with sort_utt the
batch is in DESCENDING length order (base.py:188-189), so the encoder's sort
is the identity.  Differences by design: features are memory-mapped
(np.load mmap) and the per-utterance slicing / stacking / splicing is
vectorised (frame_ops.py); the GPU hand-off (pinned buffers, async H2D on a
copy stream, lengths and labels on device, prefetch) is device_batch.py.
The reference's torch.multiprocessing preloading (num_enque) is replaced by
that prefetch thread.
"""
import math
import os
import random
import struct
from os.path import basename

import numpy as np

from .frame_ops import do_splice, slice_features, stack_frame


def librispeech_batch_rule(batch_size, min_frame_num_batch):
    """load_dataset.py:124-142 (dynamic batching thresholds)."""
    if min_frame_num_batch <= 800:
        pass
    elif min_frame_num_batch <= 1200:
        batch_size = int(batch_size / 2)
    elif min_frame_num_batch <= 1500:
        batch_size = int(batch_size / 2)
    elif min_frame_num_batch <= 1700:
        batch_size = int(batch_size / 4)
    else:
        batch_size = int(batch_size / 8)
    return max(batch_size, 1)


def load_htk(path):
    """base.py:235-258: big-endian HTK feature file -> [frames, dim] f32."""
    with open(path, 'rb') as f:
        frame_num, _, samp_size, _ = struct.unpack('>IIHH', f.read(12))
        data = np.fromfile(f, '>f4').reshape(-1, samp_size // 4)
    return data.astype(np.float32)


class DatasetBase(object):
    """df: a pandas DataFrame (or a CSV path) with frame_num / input_path /
    transcript ("i j k" label indices)."""

    def __init__(self, df, batch_size, input_freq, use_delta=False, use_double_delta=False,
                 max_epoch=None, splice=1, num_stack=1, num_skip=1, min_frame_num=40,
                 shuffle=False, sort_utt=False, reverse=False, sort_stop_epoch=None,
                 dynamic_batching=False, is_test=False, batch_rule=librispeech_batch_rule,
                 backend='pytorch'):
        import pandas as pd
        if isinstance(df, str):
            df = pd.read_csv(df)
        df = df.loc[:, ['frame_num', 'input_path', 'transcript']]
        if not is_test:                                  # load_dataset.py:110-115
            df = df[df['frame_num'] >= min_frame_num]
        if sort_utt:                                     # load_dataset.py:117-121
            df = df.sort_values(by='frame_num', ascending=not reverse)
        else:
            df = df.sort_values(by='input_path', ascending=True)
        self.df = df
        self.batch_size = batch_size
        self.input_freq = input_freq
        self.use_delta = use_delta
        self.use_double_delta = use_double_delta
        self.max_epoch = max_epoch
        self.splice = splice
        self.num_stack = num_stack
        self.num_skip = num_skip
        self.shuffle = shuffle
        self.sort_utt = sort_utt
        self.sort_stop_epoch = sort_stop_epoch
        self.dynamic_batching = dynamic_batching
        self.is_test = is_test
        self.batch_rule = batch_rule
        self.backend = backend
        self.input_size = (input_freq * (3 if use_double_delta else 2 if use_delta else 1) *
                           num_stack * splice)
        self.epoch = 0
        self.iteration = 0
        self.offset = 0
        self._epoch = 0
        self._reset()

    # ------------------------------------------------------------- iteration
    def __len__(self):
        return len(self.df)

    def __iter__(self):
        return self

    @property
    def pad_value(self):
        return -1 if not self.is_test else None

    @property
    def epoch_detail(self):
        return self.epoch + self.offset / len(self)

    @property
    def current_batch_size(self):
        return self._current_batch_size

    def _reset(self):
        self.rest = set(list(self.df.index))
        self.offset = 0

    def reset(self):
        self._reset()

    def select_batch_size(self, batch_size, min_frame_num_batch):
        if not self.dynamic_batching:
            return batch_size
        return self.batch_rule(batch_size, min_frame_num_batch)

    def sample_index(self, batch_size):
        """base.py:146-201."""
        is_new_epoch = False
        if self.sort_utt or not self.shuffle:
            if self.sort_utt:
                min_frame = self.df[self.offset:self.offset + 1]['frame_num'].values[0]
                bs = self.select_batch_size(batch_size, min_frame)
            else:
                bs = batch_size
            if len(self.rest) > bs:
                data_indices = list(self.df[self.offset:self.offset + bs].index)
                self.rest -= set(data_indices)
                self.offset += len(data_indices)
            else:
                data_indices = list(self.rest)
                self._reset()
                is_new_epoch = True
                self._epoch += 1
                if self._epoch == self.sort_stop_epoch:
                    self.sort_utt = False
                    self.shuffle = True
            data_indices = data_indices[::-1]        # descending for pytorch
        else:
            if len(self.rest) > batch_size:
                data_indices = random.sample(list(self.rest), batch_size)
                self.rest -= set(data_indices)
            else:
                data_indices = list(self.rest)
                self._reset()
                is_new_epoch = True
                self._epoch += 1
                random.shuffle(data_indices)
        return data_indices, is_new_epoch

    def __next__(self, batch_size=None):
        """base.py:76-143 (num_enque preloading: device_batch.DeviceBatches)."""
        if batch_size is None:
            batch_size = self.batch_size
        if self.max_epoch is not None and self.epoch >= self.max_epoch:
            raise StopIteration
        data_indices, is_new_epoch = self.sample_index(batch_size)
        self._current_batch_size = len(data_indices)
        batch = self.make_batch(data_indices)
        self.iteration += len(data_indices)
        if is_new_epoch:
            self.epoch += 1
        return batch, is_new_epoch

    def next(self, batch_size=None):
        return self.__next__(batch_size)

    # --------------------------------------------------------------- batches
    def load(self, path):
        ext = os.path.basename(path).split('.')[-1]
        if ext == 'npy':
            return np.load(path, mmap_mode='r')
        if ext == 'htk':
            return load_htk(path)
        raise ValueError('unknown feature file type: %s' % path)

    def features(self, path):
        """One utterance's model input (loader.py:100-141)."""
        x = slice_features(self.load(path), self.input_freq, self.use_delta,
                           self.use_double_delta)
        if self.num_stack > 1:
            x = stack_frame(x, self.num_stack, self.num_skip)
        if self.splice > 1:
            x = do_splice(x, self.splice, self.num_stack)
        return x

    def make_batch(self, data_indices, out=None):
        """loader.py:29-157.  out: optional preallocated f32 buffer (e.g. a
        pinned host tensor's numpy view) of at least B * T_max * F floats; xs
        is then a view of it."""
        rows = self.df.loc[data_indices]
        paths = np.array(rows['input_path'])
        trans = np.array(rows['transcript'])
        B = len(data_indices)
        max_frame = math.ceil(max(rows['frame_num']) / self.num_skip)
        max_label = max(len(str(t).split(' ')) for t in trans)
        if out is None:
            xs = np.zeros((B, max_frame, self.input_size), np.float32)
        else:
            xs = out.reshape(-1)[:B * max_frame * self.input_size].reshape(
                B, max_frame, self.input_size)
            xs.fill(0)
        if self.is_test:
            ys = np.array([[self.pad_value] * max_label] * B)
        else:
            ys = np.full((B, max_label), self.pad_value, np.int32)
        x_lens = np.zeros(B, np.int32)
        y_lens = np.zeros(B, np.int32)
        names = np.array([basename(p).split('.')[0] for p in paths])
        for b in range(B):
            x = self.features(paths[b])
            n = x.shape[0]
            xs[b, :n] = x
            x_lens[b] = n
            if self.is_test:
                ys[b, 0] = trans[b]
            else:
                idx = list(map(int, str(trans[b]).split(' ')))
                ys[b, :len(idx)] = idx
                y_lens[b] = len(idx)
        return {'xs': xs, 'ys': ys, 'x_lens': x_lens, 'y_lens': y_lens, 'input_names': names}

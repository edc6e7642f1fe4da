"""Per-utterance feature preparation of the reference's make_batch
(utils/dataset/loader.py:100-141): feature slicing by input_freq / delta
flags (with the pitch-column rule), frame stacking and skipping
(utils/io/inputs/frame_stacking.py) and splicing (utils/io/inputs/splicing.py),
vectorised with numpy index arithmetic (the reference loops per frame) and
reproducing the reference's index conventions exactly, quirks included:

  * stacking: T' = (T + 1) // skip output frames; the frames past the last full
    window repeat the shrinking tail window zero-padded on the right;
  * splicing: output frame t gathers source frames t - splice + i
    (i = 0..splice-1; clamped to the first / last frame), i.e. the window ends
    one frame BEFORE t, with the (freq, 3, stack) re-layout of splicing.py.
"""
import numpy as np


def slice_features(data, input_freq, use_delta, use_double_delta):
    """loader.py:100-125 (the last dim: static | delta | double delta blocks)."""
    max_input_freq = data.shape[-1] // 3
    if input_freq < max_input_freq and (input_freq - 1) % 10 == 0:
        cols = list(range(0, input_freq - 1)) + [max_input_freq]
        if use_delta:
            cols += list(range(max_input_freq, max_input_freq + input_freq - 1))
            cols += [max_input_freq * 2]
        if use_double_delta:
            cols += list(range(max_input_freq * 2, max_input_freq * 2 + input_freq - 1))
            cols += [data.shape[-1] - 1]
    else:
        cols = list(range(0, input_freq))
        if use_delta:
            cols += list(range(max_input_freq, max_input_freq + input_freq))
        if use_double_delta:
            cols += list(range(max_input_freq * 2, max_input_freq * 2 + input_freq))
    if cols == list(range(data.shape[-1])):
        return np.asarray(data, np.float32)
    return np.ascontiguousarray(np.asarray(data)[:, cols], np.float32)


def stack_frame(x, num_stack, num_skip):
    """frame_stacking.py: [T, F] -> [(T + 1) // num_skip, F * num_stack].
    Windows completed before the last frame start at k * num_skip; at the last
    frame the pending window (every frame since the last emitted start) is
    emitted and num_skip frames dropped until (T + 1) // num_skip rows exist."""
    if num_stack == 1 and num_skip == 1:
        return x
    if num_stack < num_skip:
        raise ValueError('num_skip must be less than num_stack.')
    T, F = x.shape
    Tn = (T + 1) // num_skip
    out = np.zeros((Tn, F * num_stack), np.float32)
    n_main = (T - 1 - num_stack) // num_skip + 1 if T - 1 >= num_stack else 0
    if n_main:
        idx = np.arange(n_main)[:, None] * num_skip + np.arange(num_stack)[None, :]
        out[:n_main] = x[idx].reshape(n_main, F * num_stack)
    pending = list(range(n_main * num_skip, T))
    k = n_main
    while k < Tn:
        if len(pending) > num_stack:     # the reference fails here too (row overflow)
            raise ValueError('stack_frame: pending window longer than num_stack')
        for i, f in enumerate(pending):
            out[k, F * i:F * (i + 1)] = x[f]
        k += 1
        pending = pending[num_skip:]
    return out


def do_splice(x, splice=1, num_stack=1):
    """splicing.py: [T, freq*3*stack] -> [T, freq * splice * stack * 3].
    Output frame t takes source frames t - splice + i (i < splice, clamped at
    0).  Each source frame is re-laid (freq, 3, stack) -> (stack, freq, 3) and
    written at rows [i, i + stack) of a (splice * stack)-row block, so for
    stack > 1 later frames overwrite earlier ones and rows past
    splice + stack - 1 stay zero, exactly as the reference's slice does."""
    if splice == 1:
        return x
    T, D = x.shape
    assert D % 3 == 0
    freq = (D // 3) // num_stack
    R = splice * num_stack
    src = np.clip(np.arange(T)[:, None] + np.arange(splice)[None, :] - splice, 0, T - 1)
    frames = x[src].reshape(T, splice, freq, 3, num_stack).transpose(0, 1, 4, 2, 3)
    block = np.zeros((T, R, freq, 3), np.float32)                 # (T, rows, freq, 3)
    for j in range(min(R, splice + num_stack - 1)):
        i = min(j, splice - 1)
        block[:, j] = frames[:, i, j - i]
    return np.ascontiguousarray(block.transpose(0, 2, 1, 3).reshape(T, freq * R * 3), np.float32)

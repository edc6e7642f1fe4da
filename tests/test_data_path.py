"""The data path: DatasetBase batch order, dynamic
batch halving, padding, feature slicing / stacking / splicing against a
fixture recorded from the reference's own DatasetBase + LibriSpeech Dataset
(tests/golden/make_golden.py case_loader); the device hand-off
(utils/dataset/device_batch.py) on the GPU: the device batch equals the host
batch, and one train_step runs from it."""
import numpy as np
import pandas as pd
import pytest
import torch

from conftest import golden
from pytorch_end2end_speech_recognition_amd.utils.dataset import frame_ops
from pytorch_end2end_speech_recognition_amd.utils.dataset.loader import DatasetBase


def _dataset(d, tmp_path, tag):
    n = len(d['df_frame_num'])
    paths = []
    for i in range(n):
        p = str(tmp_path / ('utt%03d.npy' % i))
        np.save(p, d['feat/utt%03d' % i])
        paths.append(p)
    df = pd.DataFrame({'frame_num': d['df_frame_num'], 'input_path': paths,
                       'transcript': [str(t) for t in d['df_transcript']]})
    bs, sort_utt, reverse, dyn, freq, delta, dd, stack, skip, splice = \
        [int(v) for v in d['spec/' + tag]]
    return DatasetBase(df, bs, freq, use_delta=bool(delta), use_double_delta=bool(dd),
                       max_epoch=2, splice=splice, num_stack=stack, num_skip=skip,
                       sort_utt=bool(sort_utt), reverse=bool(reverse),
                       dynamic_batching=bool(dyn))


@pytest.mark.parametrize('tag', ['a', 'b', 'c'])
def test_batches_match_reference(tag, tmp_path):
    d = golden('loader')
    ds = _dataset(d, tmp_path, tag)
    nb = int(d['%s/n_batches' % tag][0])
    k = 0
    for batch, new_epoch in ds:
        pre = '%s/%d/' % (tag, k)
        names = [int(s[3:]) for s in batch['input_names']]
        np.testing.assert_array_equal(names, d[pre + 'utts'], err_msg=pre)
        assert int(new_epoch) == int(d[pre + 'new_epoch'][0])
        for key in ('xs', 'ys', 'x_lens', 'y_lens'):
            np.testing.assert_array_equal(batch[key], d[pre + key], err_msg=pre + key)
        k += 1
    assert k == nb


def test_frame_ops_match_reference():
    d = golden('loader')
    x = d['stack_in']
    for key in d.files:
        if key.startswith('stack/'):
            st, sk = map(int, key[6:].split('_'))
            np.testing.assert_array_equal(frame_ops.stack_frame(x, st, sk), d[key], err_msg=key)
        if key.startswith('splice/'):
            sp, ns = map(int, key[7:].split('_'))
            np.testing.assert_array_equal(frame_ops.do_splice(x[:, :12 * ns], sp, ns), d[key],
                                          err_msg=key)


@pytest.mark.gpu
def test_device_batches_and_train_step(tmp_path, cuda_dev):
    from pytorch_end2end_speech_recognition_amd import native_ops
    from pytorch_end2end_speech_recognition_amd.models.pytorch_v3.ctc.ctc import CTC
    from pytorch_end2end_speech_recognition_amd.utils.dataset.device_batch import DeviceBatches
    from pytorch_end2end_speech_recognition_amd.utils.training.training_loop import train_step
    d = golden('loader')
    ref = _dataset(d, tmp_path, 'a')
    it = DeviceBatches(_dataset(d, tmp_path, 'a'), cuda_dev, depth=2)
    native_ops.set_compute_dtype('fp32')
    torch.manual_seed(1623)
    model = CTC(input_size=123, encoder_type='lstm', encoder_bidirectional=True,
                encoder_num_units=16, encoder_num_proj=0, encoder_num_layers=2, fc_list=[],
                dropout_input=0, dropout_encoder=0, num_classes=29, parameter_init=0.1)
    model.set_cuda()
    model.set_optimizer('adam', 1e-3, weight_decay=1e-6, lr_schedule=False)
    n = 0
    try:
        for (db, e1), (hb, e2) in zip(it, ref):
            assert e1 == e2
            torch.cuda.synchronize()
            np.testing.assert_array_equal(db['xs'].cpu().numpy(), hb['xs'])
            np.testing.assert_array_equal(db['x_lens_d'].cpu().numpy(), hb['x_lens'])
            np.testing.assert_array_equal(db['y_lens_d'].cpu().numpy(), hb['y_lens'])
            flat = np.concatenate([hb['ys'][b, :hb['y_lens'][b]] + 1 for b in range(len(hb['ys']))])
            np.testing.assert_array_equal(db['labels_d'].cpu().numpy(), flat)
            model, lv = train_step(model, db, clip_grad_norm=5.0)
            assert np.isfinite(lv)
            n += 1
    finally:
        it.close()
    assert n == int(d['a/n_batches'][0])

"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

This package restates the reference algorithm for the hot path
(TheCacophonyProject/audio-training: custommel.py, tfdataset.py normalize /
mix_up / raw_to_mel, predict_utils.get_spect, tfpcen.py, resnet/wr_resnet*.py,
audiomodel.loss / optimizer) on the CPU so that the HIP path can be checked.

Only `tests/`, `__graft_entry__.smoke()` and the `cpu_baseline` leg of
`bench.py` may import it, and only as the checker / the reported CPU baseline.
The product path (`audio-training_amd/`) never imports it and fails loudly when
its HIP library is missing.

Parity pinning:
  * `mel_f` / `mel_spec` are pinned bit-for-bit against golden vectors produced
    by the reference `custommel.py` itself (oracle/gen_golden.py ->
    tests/golden/mel_f_*.npz, mel_spec_p*.npz).
  * The streaming path's index work -- identifytracks.merge_signals /
    get_tracks_from_signals / Signal / get_end's chunk scan and
    predict_utils.load_samples' window cutting -- is pinned bit-for-bit
    against tests/golden/tracks_golden.npz, produced by the reference modules
    themselves (oracle/gen_golden_tracks.py, stub librosa / cv2 / tensorflow
    imports that those functions never call).
  * STFT (tf.signal.stft pad_end, librosa.stft center), PCEN, LME, Keras layer
    semantics and Adam live in third-party libraries (tensorflow, tfp,
    librosa, keras -- unpinned in requirements.txt:1-13) that are absent from
    this image; they are restated from their published definitions and are
    "parity unpinned" beyond the golden mel filterbank.
"""

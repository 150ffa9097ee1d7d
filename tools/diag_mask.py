"""Masked-stream vs default-stream results of mel and embed (diagnostic)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
import torch  # noqa: E402

from heybuddy.embedding_graph import WINDOW_STARTS  # noqa: E402
from heybuddy.embeddings import embed_plan  # noqa: E402
from heybuddy.kernels import embed_clips, mel_frames  # noqa: E402
from heybuddy.pipeline import make_streams  # noqa: E402
from heybuddy.spectrogram import default_mel_plan  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(3)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
clips = torch.randn((n, 24000), generator=g, device=dev) * 0.1
mplan = default_mel_plan(dev, 32767.0)
eplan = embed_plan(dev, WINDOW_STARTS)
mel_ref = mel_frames(clips, mplan, 141).clone()
emb_ref = embed_clips(mel_ref, eplan).clone()
emb_ref2 = embed_clips(mel_ref, eplan).clone()
print("default stream repeat equal:", torch.equal(emb_ref, emb_ref2))
fs, ts, keep = make_streams(dev, "split:64")
for name, st in (("feature(192)", fs), ("train(64)", ts)):
    st.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(st):
        mel = mel_frames(clips, mplan, 141)
        emb = embed_clips(mel_ref, eplan)
    torch.cuda.current_stream(dev).wait_stream(st)
    torch.cuda.synchronize()
    dm = (mel - mel_ref).abs().max().item()
    de = (emb - emb_ref).abs()
    bad = (de.flatten(1).max(1).values > 0).nonzero().flatten().tolist()
    print(f"{name}: mel max|d| {dm:.3e}; embed max|d| {de.max().item():.3e}, clips differing {len(bad)} "
          f"{bad[:10]}, rel {(de.max() / emb_ref.abs().max()).item():.3e}")

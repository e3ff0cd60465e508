"""A throughput batch whose upload is staged and copied in pieces (cedar_eval.hip dev_batch_upload:
>= 64 MB to stage, one H2D copy per 16 MB piece as soon as it is staged) decides every request as
the same requests do in batches small enough for the one-copy upload."""
import pytest

import cedargpu
from cedargpu import synth

from test_gpu_parity import ctx  # noqa: F401  (module fixture)

pytestmark = pytest.mark.gpu


def test_piecewise_upload_matches_one_copy_uploads(ctx):  # noqa: F811
    pop = synth.Population(seed=7, n_users=3000, n_groups=300, dag_depth=6)
    img = cedargpu.build_image([cedargpu.MemoryStore("c3.cedar", synth.abac_policies(2000, seed=5, pop=pop))],
                               epoch=971, entities=pop.static_entities())
    ctx.load(img, 971)
    sars = synth.random_sars(200_000, seed=77, pop=pop)

    def run(part):
        b = ctx.batch()
        b.add_sar_json(synth.sars_json(part).encode())
        b.submit()
        b.wait()
        io = b.io()
        out = [b.authz(i) for i in range(len(part))]
        b.close()
        return out, io["h2d_bytes"]

    whole, h2d = run(sars)
    assert h2d >= 64 << 20, "the batch must take the piecewise upload"
    parts = []
    for k in range(0, len(sars), 40_000):
        got, h = run(sars[k:k + 40_000])
        assert h < 64 << 20
        parts += got
    assert whole == parts

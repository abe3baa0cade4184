

def test_hash_to_g1_many_matches_scalar_path():
    """The batched BLS map (native square roots of the first candidates of
    every message) gives the same points as the one-message map."""
    import os

    from drynx_amd.crypto import bls

    msgs = [os.urandom(32) for _ in range(12)] + [b""]
    assert bls.hash_to_g1_many(msgs) == [bls.hash_to_g1(m) for m in msgs]
    assert bls.hash_to_g1_many(msgs, tries=1) == [bls.hash_to_g1(m) for m in msgs]

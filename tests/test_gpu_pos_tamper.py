"""GPU: the reference's fault-injection test, test_file_verification_rejects_bad_proofs
(proof-of-storage/src/networking/tests.rs:696-780), without the network.  The server stores the
reference's test.txt at 4/8 columns (FileHandler); a proof request re-encodes the server's raw
file and serves the client's columns with paths (convert_file_data_to_commit, ColumnsWithPath);
the client checks them against the root it kept at upload (client_online_verify_column_paths).
After two bytes of the server's raw file are overwritten at the ChaCha8(1337) offset, the next
request must fail, and so must the server's own verify_all_files_agree."""
import os

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
TEST_TXT = os.path.join(HERE, "golden", "pos_test.txt")


def test_tampered_server_file_fails_client_verification(gpu, oracle, tmp_path):
    from lcpc_proof_of_storage_amd import pos, pos_files
    data = open(TEST_TXT, "rb").read()
    src = tmp_path / "test.txt"
    src.write_bytes(data)
    fh = pos_files.FileHandler.create_from_unencoded_file("01TAMPERTEST00000000000000", str(src), 4, 8,
                                                          directory=str(tmp_path / "files"))
    root = fh.get_commit_root()                       # what the client keeps after upload
    n_cols = pos.get_PoS_soudness_n_cols(4, 8)

    def request_proof(seed):
        cols = pos.get_column_indicies_from_random_seed(seed, n_cols, 8)
        with open(fh.get_raw_file_handle(), "rb") as f:
            field = pos.convert_byte_vec_to_field_elements_vec(f.read())
        served = pos.convert_file_data_to_commit(field, pos.ColumnsWithPath(cols), pos.Specified(4, 8))
        pos.client_online_verify_column_paths(root, cols, served)

    request_proof(1)                                  # the honest server passes
    rng = oracle.ChaCha(seed_u64=1337, rounds=8)      # ChaCha8Rng::seed_from_u64(1337)
    seek = rng.next_u32() % (len(data) - 2)
    new = rng.fill_bytes(2)
    with open(fh.get_raw_file_handle(), "r+b") as f:
        f.seek(seek)
        old = f.read(2)
        f.seek(seek)
        f.write(new)
    assert old != new
    with pytest.raises(gpu.VerifierError):
        request_proof(2)
    with pytest.raises(AssertionError):
        fh.verify_all_files_agree()
    fh.delete_all_files()

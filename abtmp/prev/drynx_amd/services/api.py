"""Querier/client API.

Reference: services/api.go (``NewDrynxClient`` :39 — keypair + decryption
table of 10000 entries; ``GenerateSurveyQuery`` :58-102; ``SendSurveyQuery``
:105-133) and services/api_skipchain.go (``SendSurveyQueryToVNs`` :16,
``SendEndVerification`` :30, ``SendGetLatestBlock`` :44, ``SendGetGenesis``
:61, ``SendGetBlock`` :71, ``SendGetProofs`` :86, ``SendCloseDB`` :98).

The client talks to an entry point: an in-process ``DrynxNode`` (rank 0 of a
local cluster) or a ``RemoteNode`` (TCP control plane to a running server,
see services/server.py).
"""
from __future__ import annotations

from ..crypto import elgamal as eg
from ..ops import encoding as enc
from ..query import (LogisticRegressionParameters, Operation, Query, QueryDiffP, QueryDPDataGen, QueryIVSigs, Roster,
                     SurveyQuery, new_survey_id)
from ..utils import timers


class DrynxClient:
    def __init__(self, entry_point, keypair: eg.KeyPair | None = None, decrypt_bound: int = 10000, device="cpu"):
        self.entry = entry_point
        self.keypair = keypair or eg.KeyPair.generate()
        self.public = self.keypair.public
        self.device = device
        self.decrypt_bound = decrypt_bound
        self._table = None
        self.last_plaintexts: list = []  # the decrypted aggregate of the last logistic-regression query, per group

    @property
    def table(self) -> eg.DecryptionTable:
        """CreateDecryptionTable(limit) — built lazily on the client's device."""
        if self._table is None or self._table.bound != self.decrypt_bound:
            self._table = eg.decryption_table(self.decrypt_bound, self.device)
        return self._table

    # ------------------------------------------------------------------ query building
    def generate_survey_query(self, roster_servers: Roster, roster_vns: Roster | None, dp_to_server: dict,
                              id_to_public: dict, survey_id: str | None, operation: Operation, ranges, ps,
                              proofs: int, obfuscation: bool, thresholds, diffp: QueryDiffP | None = None,
                              dpdatagen: QueryDPDataGen | None = None, cutting_factor: int = 0,
                              verification_sharding: int = 0, range_proof_mode: int = 0) -> SurveyQuery:
        """GenerateSurveyQuery; thresholds = [general, aggregation, range, obfuscation, keyswitch] (api.go:79-83)."""
        sq = SurveyQuery(
            SurveyID=survey_id or new_survey_id(),
            RosterServers=roster_servers,
            ClientPubKey=self.public,
            IntraMessage=False,
            ServerToDP=dp_to_server,
            Query=Query(Operation=operation, Ranges=ranges, Proofs=proofs, Obfuscation=obfuscation,
                        DiffP=diffp or QueryDiffP(), DPDataGen=dpdatagen or QueryDPDataGen(),
                        IVSigs=QueryIVSigs(InputValidationSigs=ps,
                                           InputValidationSize1=len(ps) if ps else 0,
                                           InputValidationSize2=len(ps[0]) if ps else 0),
                        RosterVNs=roster_vns, CuttingFactor=cutting_factor),
            IDtoPublic=id_to_public,
            Threshold=thresholds[0], AggregationProofThreshold=thresholds[1], RangeProofThreshold=thresholds[2],
            ObfuscationProofThreshold=thresholds[3], KeySwitchingProofThreshold=thresholds[4],
            VerificationSharding=verification_sharding,
            RangeProofMode=range_proof_mode,
        )
        return sq

    # ------------------------------------------------------------------ execution
    def send_survey_query(self, sq: SurveyQuery):
        """SendSurveyQuery: run the survey, decode every group.  Returns
        (group keys, list of decoded float vectors, SurveyResult)."""
        op = sq.Query.Operation

        def decode_all(partial):
            groups, values = [], []
            self.last_plaintexts = []
            with timers.timed("Decode"):
                for g, cv in enumerate(partial.groups()):
                    groups.append(str(g))
                    values.append(self.decode(cv.to(self.device), op))
            return groups, values

        # decoding overlaps the VNs' proof verification (own thread + stream)
        res = self.entry.run_survey(sq, on_result=decode_all)
        groups, values = res.client_out
        return groups, values, res

    def decode(self, cv: eg.CipherVector, op: Operation):
        if op.NameOp == "logistic regression":
            with timers.timed("Decryption"):
                vals = [int(v) for v in eg.decrypt_auto(self.keypair.secret, cv, self.decrypt_bound).cpu().tolist()]
            self.last_plaintexts.append(vals)
            from ..models.logistic_regression import decode_logistic_regression_values

            return decode_logistic_regression_values(vals, op.LRParameters)
        return enc.decode(cv, self.keypair.secret, op, self.table)

    # ------------------------------------------------------------------ VN / skipchain calls
    def send_survey_query_to_vns(self, sq: SurveyQuery):
        """SendSurveyQueryToVNs (api_skipchain.go:16): announce the survey to the
        VNs before running it (expected proof counts, ledger, chain)."""
        return self.entry.register_vn_survey(sq)

    def send_end_verification(self, vn_id: str, survey_id: str, timeout: float | None = 3600.0):
        """SendEndVerification (api_skipchain.go:30): blocks until the VNs have
        verified every proof of the survey and the root VN appended its block
        (EndVerificationChannel, service_skipchain.go:158-166); returns it, or
        None on timeout.  Callable before or while the survey runs."""
        return self.entry.wait_end_verification(survey_id, timeout)

    def send_get_latest_block(self, vn_id: str, sb=None):
        """SendGetLatestBlock (api_skipchain.go:44): the VN's head, or -- given a
        known block ``sb`` -- the end of the verified update chain from it."""
        return self.entry.get_latest_block(vn_id, sb) if sb is not None else self.entry.get_latest_block(vn_id)

    def send_get_genesis(self, vn_id: str):
        return self.entry.get_genesis(vn_id)

    def send_get_block(self, vn_id: str, survey_id: str):
        return self.entry.get_block(vn_id, survey_id)

    def send_get_proofs(self, vn_id: str, survey_id: str) -> dict:
        return self.entry.get_proofs(vn_id, survey_id)

    def send_close_db(self, vn_id: str, remove: bool = False):
        return self.entry.close_db(vn_id, remove)


def lr_parameters(**kw) -> LogisticRegressionParameters:
    return LogisticRegressionParameters(**kw)

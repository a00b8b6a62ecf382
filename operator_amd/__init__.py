"""operator_amd — MI355X-native pod-failure analysis operator.

Same Podmortem / PatternLibrary / AIProvider API and reconcile semantics as
podmortem/operator, with the reference's two remote hops (log-parser,
ai-interface) pulled on-node as GPU stages: a hand-written CDNA4 Aho-Corasick
log scan and a local Llama explanation engine on hand-written HIP kernels.
See README.md and SURVEY.md.
"""
__version__ = "0.1.0"

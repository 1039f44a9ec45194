"""cron-operator-amd: a from-scratch cron operator for scheduled ML training jobs.

Same API and behaviour as AliyunContainerService/cron-operator (``apps.kubedl.io/v1alpha1``
``Cron``), re-designed: asyncio control plane with native C++ hot paths (cron engine,
JSON-tree ops), informer-cached child listing, an in-process fake apiserver for tests,
and PyTorch-ROCm/RCCL example payloads for MI355X nodes.  See README.md and SURVEY.md.
"""
__version__ = "0.3.0"

"""Reference module path of the dashboard REST client (``p2pfl/management/p2pfl_web_services.py``);
the implementation is :mod:`myfyp_amd.management.web_services`."""

from myfyp_amd.management.web_services import P2pflWebServices, P2pflWebServicesError

__all__ = ["P2pflWebServices", "P2pflWebServicesError"]

"""Authentication: local passwords, LDAP, OAuth2 SSO, registration workflows, reserved names.

Reference: config_settings/auth.py, registration.py, api/users/views.py, sso/, libs/blacklist.py.
"""
from polyaxon_amd.auth.accounts import Accounts, AuthError  # noqa: F401
from polyaxon_amd.auth.passwords import (RESERVED_NAMES, check_password, hash_password,  # noqa: F401
                                         validate_name)

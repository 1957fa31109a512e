"""FaaS entry points of the aggregator function, over the in-memory stores.

Restates, for the engine:
  functions/aggregator_functions/openfaas/aggregator/aggregator/handler.py:16-28   handle(event, context)
  functions/aggregator_functions/openwhisk/aggregator/main.py:12-24                main(request)
and the provider decorators they are wrapped in (fedless/common/providers.py):
  create_http_success_response      :16-22   {"statusCode": 200, "body": result.json(), "headers": ...}
  format_exception_for_user         :25-31   {"errorMessage", "errorType", "details"}
  create_http_user_error_response   :34-40   the same with statusCode 400
  openfaas_action_handler           :156-177 ValidationError / AggregationError -> 400
  openwhisk_action_handler          :180-218 "__ow_" web-action keys stripped, plain params put
                                             under "body", a str/bytes body parsed as JSON or
                                             base64(JSON); decode errors -> 400 as well

The request is the reference's AggregatorFunctionParams JSON. Its MongoDB
`database` section is accepted and not used: the handler reads results from,
and saves the new global model into, the stores the entry point was built
with. Global evaluation (`test_data`) is out of scope and answers 400.
"""
from __future__ import annotations

import base64
import binascii
import json
import traceback
from json import JSONDecodeError
from typing import Callable, Dict, Optional

from pydantic import ValidationError

from .aggregator.exceptions import AggregationError
from .common.models import AggregatorFunctionParams
from .handler import default_aggregation_handler
from .store import InMemoryClientResultStore, InMemoryParameterStore

_JSON = {"Content-Type": "application/json"}


def create_http_success_response(body: str, status: int = 200) -> Dict:
    """providers.py:16-22"""
    return {"statusCode": status, "body": body, "headers": dict(_JSON)}


def format_exception_for_user(exception: Exception) -> Dict:
    """providers.py:25-31"""
    return {"errorMessage": str(exception), "errorType": exception.__class__.__name__,
            "details": traceback.format_exc()}


def create_http_user_error_response(exception: Exception, status: int = 400) -> Dict:
    """providers.py:34-40"""
    return {"statusCode": status, "body": json.dumps(format_exception_for_user(exception)), "headers": dict(_JSON)}


def _run(config: AggregatorFunctionParams, result_store, parameter_store, device, devices=None) -> str:
    result = default_aggregation_handler(
        session_id=config.session_id, round_id=config.round_id, result_store=result_store,
        parameter_store=parameter_store, serializer=config.serializer, test_data=config.test_data,
        aggregation_strategy=config.aggregation_strategy,
        aggregation_hyper_params=config.aggregation_hyper_params, device=device, devices=devices)
    return json.dumps(result.model_dump(mode="json"))  # pydantic-v1 .json() layout (providers.py:172)


def make_openfaas_handler(result_store: InMemoryClientResultStore, parameter_store: InMemoryParameterStore,
                          device=None, devices=None) -> Callable:
    """handle(event, context) of the OpenFaaS aggregator (handler.py:16-28):
    event.body is the AggregatorFunctionParams JSON.  devices: fold on several
    GPUs of the function's process (one column bucket each)."""

    def handle(event, context=None) -> Dict:
        try:
            config = AggregatorFunctionParams.model_validate_json(event.body)
            return create_http_success_response(_run(config, result_store, parameter_store, device, devices))
        except (ValidationError, AggregationError) as e:
            return create_http_user_error_response(e)

    return handle


def make_openwhisk_main(result_store: InMemoryClientResultStore, parameter_store: InMemoryParameterStore,
                        device=None, devices=None) -> Callable:
    """main(request) of the OpenWhisk aggregator (main.py:12-24) with the
    openwhisk_action_handler parameter handling (providers.py:180-218)."""

    def main(params: Dict) -> Dict:
        if any(k.startswith("__ow_") for k in params):  # web action: strip the prefix
            params = {(k[len("__ow_"):] if k.startswith("__ow_") else k): v for k, v in params.items()}
        else:
            params = {"body": params}
        try:
            body = params["body"]
            if isinstance(body, (str, bytes)):  # OpenWhisk sometimes base64-encodes the body
                try:
                    body = json.loads(body)
                except JSONDecodeError:
                    body = json.loads(base64.b64decode(body))
            config = AggregatorFunctionParams.model_validate(body)
            return create_http_success_response(_run(config, result_store, parameter_store, device, devices))
        except (ValidationError, AggregationError, JSONDecodeError, binascii.Error) as e:
            return create_http_user_error_response(e)

    return main


class Event:
    """Minimal stand-in for the OpenFaaS request object (only .body is read)."""

    def __init__(self, body, headers: Optional[Dict] = None):
        self.body = body
        self.headers = headers or {}

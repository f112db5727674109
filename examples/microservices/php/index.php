<?php
echo "Hello from the php microservice\n";

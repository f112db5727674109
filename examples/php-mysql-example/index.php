<?php
// Connects to the mysql container of the same pod using the env vars from chart/values.yaml.
$host = getenv('DB_HOST') ?: '127.0.0.1';
$conn = @new mysqli($host, getenv('DB_USER'), getenv('DB_PASSWORD'), getenv('DB_NAME'));
if ($conn->connect_error) {
    echo "Waiting for the database: " . $conn->connect_error . "\n";
} else {
    echo "Connected to MySQL " . $conn->server_info . "\n";
}
